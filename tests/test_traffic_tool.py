"""tools/traffic.py (round 6): PMC bytes counted over the timed graph replays only -- the pre-capture
segment (planning forward, autotune candidates) is dropped, per-kernel dispatch counts are reconciled,
and the launch list must match the kernel trace's timeline name for name."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TOOL = os.path.join(os.path.dirname(HERE), "tools", "traffic.py")
FIELDS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
          "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
          "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
FWD = ["void yxh::stem_s2<bool _Accum, 32, true>(yxh::Stem2Params, int, int, int)",
       "_ZN3yxh7conv_wsIDF16bLi128ELi1ELi16ELi4ELi128ELi4ELi1ELi1ELi1ELb0ELi0ELi0ELi0ELi128ELb0EEEvNS_10ConvParamsEiiiii",
       "_ZN3yxh7conv_wsIDF16bLi128ELi1ELi16ELi4ELi128ELi4ELi1ELi1ELi1ELb0ELi0ELi0ELi0ELi128ELb0EEEvNS_10ConvParamsEiiiii",
       "_ZN3yxh10head_pred2IDF16bLi128ELi5EEEv13yxh_head_desc"]


def write_pass(path, counter, value_of):
    os.makedirs(path, exist_ok=True)
    rows, did = [], 0

    def add(name, v):
        nonlocal did
        did += 1
        rows.append(dict.fromkeys(FIELDS, 0) | {"Dispatch_Id": did, "Kernel_Name": name, "Counter_Name": counter,
                                                "Counter_Value": v})
    add("__amd_rocclr_copyBuffer", 5.0)
    # the eager planning forward: the stem, then autotune candidates of other families
    add(FWD[0], 100.0)
    for _ in range(7):
        add("_ZN3yxh10conv_igemmIDF16bLi64EEEvNS_10ConvParamsE", 1000.0)
    for _ in range(3):  # timed replays, each followed by the NMS kernels
        for n in FWD:
            add(n, value_of(n))
        add("yxh::pp_filter_scored(float*, float4 const*, int, int, float, yxh::PPWork)", 7.0)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, FIELDS)
        w.writeheader()
        w.writerows(rows)


def timeline(path, names):
    with open(path, "w") as f:
        f.write("  #    start      end     dur    gap ovl  kernel\n")
        for i, n in enumerate(names):
            short = n.split("(")[0].replace("void ", "")[:70]
            f.write(f"{i:3d} {0.0:8.1f} {1.0:8.1f} {1.0:7.1f} {0.0:6.1f}   0  {short}\n")
        f.write("span 1.0 us\n")


def run(tmp_path, tl_names, replays=3):
    vals = {FWD[0]: 10.0, FWD[1]: 20.0, FWD[3]: 40.0}
    write_pass(str(tmp_path / "p_FETCH_SIZE"), "FETCH_SIZE", lambda n: vals[n])
    write_pass(str(tmp_path / "p_WRITE_SIZE"), "WRITE_SIZE", lambda n: vals[n] / 2)
    timeline(str(tmp_path / "tl.txt"), tl_names)
    out = tmp_path / "t.json"
    r = subprocess.run([sys.executable, TOOL, str(tmp_path / "p"), str(out), "--replays", str(replays),
                        "--timeline", str(tmp_path / "tl.txt")], capture_output=True, text=True)
    return r, out


def test_counts_only_the_timed_replays(tmp_path):
    r, out = run(tmp_path, FWD)
    assert r.returncode == 0, r.stderr
    d = json.load(open(out))
    per_fwd_fetch = 10 + 20 + 20 + 40  # KiB per replay; the planning segment's 7 conv_igemm are not counted
    assert d["forwards"] == 3 and d["launches_per_forward"] == 4
    assert d["hbm_read_bytes_per_forward"] == 2 * per_fwd_fetch * 1024  # FETCH_SIZE x2 (gfx950)
    assert d["hbm_write_bytes_per_forward"] == per_fwd_fetch / 2 * 1024
    assert d["dispatch_counts_per_kernel"][FWD[1]] == [2, 6]
    assert d["timeline_check"].startswith("4 launches per forward")


def test_timeline_mismatch_and_too_many_replays_fail(tmp_path):
    r, _ = run(tmp_path, FWD[:3])  # the trace's forward lacks the head launch
    assert r.returncode != 0 and "timeline" in r.stderr
    r, _ = run(tmp_path, FWD, replays=4)
    assert r.returncode != 0 and "trailing replays" in r.stderr

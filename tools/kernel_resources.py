"""Per-kernel resource usage of the built libyoloxhip.so (gfx950 code objects): VGPR / AGPR /
SGPR counts, LDS bytes and private-segment (scratch) bytes from the code-object metadata.

The .hip_fatbin section of a hipcc-linked shared library is the concatenation of one clang
offload bundle per translation unit; each is unbundled and its gfx950 ELF's AMDGPU metadata
note read with llvm-readelf.  Used by tests/test_native_lib.py (no shipped kernel may spill to
scratch) and by hand: python tools/kernel_resources.py [--spills]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd", "yolox_amd", "_lib",
                   "libyoloxhip.so")


def kernels(lib: str = LIB) -> dict:
    """name -> {vgpr, agpr, sgpr, lds, scratch} for every gfx950 kernel in ``lib``."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "x.so")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            part = os.path.join(td, f"b{i}.bin")
            with open(part, "wb") as f:
                f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(td, f"co{i}.o")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                               capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            # one YAML map per kernel, its keys sorted: .agpr_count and .group_segment_fixed_size come
            # BEFORE .name, so a record starts at its "- ." line and is filed under its name at the end
            rec, name = None, None
            def flush():
                if rec is not None and name:
                    out.setdefault(name, {}).update(rec)
            for line in notes.splitlines():
                t = line.strip()
                m = re.match(r"^(-?)\s*\.(\w+):\s*(.*)$", t)
                if not m:
                    continue
                item, key, val = m.group(1), m.group(2), m.group(3).strip()
                if item and key != "name" and key != "address_space" and (rec is None or key == "agpr_count"):
                    flush()
                    rec, name = {}, None
                if rec is None:
                    continue
                if key == "name" and val.startswith("_Z"):
                    name = val
                elif key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
                             "private_segment_fixed_size"):
                    short = {"vgpr_count": "vgpr", "agpr_count": "agpr", "sgpr_count": "sgpr",
                             "group_segment_fixed_size": "lds", "private_segment_fixed_size": "scratch"}[key]
                    rec[short] = int(val)
            flush()
    return out


def main():
    ks = kernels()
    spills = {k: v for k, v in ks.items() if v.get("scratch", 0) > 0}
    if "--spills" in sys.argv:
        for k, v in sorted(spills.items()):
            print(v["scratch"], k)
        print(f"{len(spills)} of {len(ks)} kernels use scratch")
        return 1 if spills else 0
    for k, v in sorted(ks.items()):
        print(v.get("vgpr"), v.get("agpr"), v.get("sgpr"), v.get("lds"), v.get("scratch"), k)
    return 0


if __name__ == "__main__":
    sys.exit(main())

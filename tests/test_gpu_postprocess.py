"""Device post-processing (yxh_postprocess) vs the C oracle: bit-exact.

The same fp32 [B, A, 5+C] prediction goes to both; keep indices, labels, boxes and
confidences must be identical, as must the in-place xyxy conversion.  Covers both
torchvision batched_nms branches (coordinate trick / per-class), class-agnostic
NMS, empty images, all-filtered batches, score ties and dense overlaps.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def run_both(oracle, pred: np.ndarray, C: int, conf: float, nms: float, agnostic=False, vanilla=4000):
    from yolox_amd.utils.boxes import postprocess
    p_gpu = torch.from_numpy(pred.copy()).cuda()
    got = postprocess(p_gpu, C, conf, nms, agnostic, vanilla_numel=vanilla)
    p_cpu = pred.copy()
    want = oracle.postprocess(p_cpu, C, conf, nms, agnostic, vanilla_numel=vanilla)
    np.testing.assert_array_equal(p_gpu.cpu().numpy(), p_cpu)  # in-place xyxy
    assert len(got) == len(want)
    for g, w in zip(got, want):
        if w is None:
            assert g is None
        else:
            assert g is not None
            np.testing.assert_array_equal(g.cpu().numpy(), w)
    return want


def synthetic_pred(B, A, C, seed, dense=False):
    rng = np.random.default_rng(seed)
    pred = np.zeros((B, A, 5 + C), np.float32)
    span = 60 if dense else 600
    pred[..., 0:2] = rng.uniform(20, 20 + span, (B, A, 2))
    pred[..., 2:4] = rng.uniform(4, 120, (B, A, 2))
    pred[..., 4] = rng.uniform(0, 1, (B, A))
    pred[..., 5:] = rng.uniform(0, 1, (B, A, C)) ** 3
    return pred


@pytest.mark.parametrize("conf", [0.01, 0.3, 0.65])
@pytest.mark.parametrize("vanilla", [4000, 0])
def test_reference_fixture_prediction(oracle, golden, conf, vanilla):
    pred = golden("postprocess_pre_nms.npz")["prediction"]
    run_both(oracle, pred, 80, conf, 0.65, vanilla=vanilla)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("dense", [False, True])
def test_random_predictions_both_branches(oracle, seed, dense):
    pred = synthetic_pred(3, 2100, 80, seed, dense)
    for conf in (0.05, 0.25):  # ~1900 / ~700 candidates: vanilla and trick branches
        run_both(oracle, pred, 80, conf, 0.45)
        run_both(oracle, pred, 80, conf, 0.65, agnostic=True)


def test_full_640_anchor_set_low_conf(oracle):
    """8400 anchors, conf 0.01: thousands of candidates (eval regime)."""
    pred = synthetic_pred(2, 8400, 80, 7, dense=True)
    want = run_both(oracle, pred, 80, 0.01, 0.65)
    assert sum(len(w) for w in want if w is not None) > 100


def test_empty_and_filtered(oracle):
    pred = synthetic_pred(3, 336, 80, 1)
    pred[1, :, 4] = 0.0  # image 1: nothing passes
    run_both(oracle, pred, 80, 0.3, 0.45)
    want = run_both(oracle, pred, 80, 1.5, 0.45)  # nothing anywhere
    assert all(w is None for w in want)


def test_score_ties_are_resolved_by_anchor_order(oracle):
    pred = synthetic_pred(1, 500, 4, 3, dense=True)
    pred[..., 4] = 0.5
    pred[..., 5:] = 0.0
    pred[0, :, 5 + 2] = 0.8  # every anchor: identical score, same class
    run_both(oracle, pred, 4, 0.1, 0.3)
    run_both(oracle, pred, 4, 0.1, 0.3, vanilla=0)


@pytest.mark.parametrize("C", [80, 7, 3, 1])
def test_class_argmax_ties_across_quarters(oracle, C):
    """The filter's class argmax runs as four partial scans + lane shuffles: equal maxima
    in different quarters (and -inf / all-equal rows) must give the serial first maximum,
    as the oracle's strict '>' scan (torch.max on the CPU tensor) does."""
    pred = synthetic_pred(2, 640, C, 13, dense=True)
    pred[..., 4] = 0.9
    q = max(1, (C + 3) // 4)
    for a in range(0, 640, 5):  # same maximum in the first class of every quarter
        pred[:, a, 5:] = 0.1
        for k in range(0, C, q):
            pred[:, a, 5 + k] = 0.7
    pred[:, 1::7, 5:] = 0.25  # all classes equal
    pred[:, 3::11, 5:] = -np.inf  # scores below conf: filtered
    pred[:, 2::13, 5 + C - 1] = 0.95  # the last class wins outright
    run_both(oracle, pred, C, 0.05, 0.5)
    run_both(oracle, pred, C, 0.05, 0.5, agnostic=True)


def test_filter_done_event_lets_the_producer_overwrite_pred(oracle):
    """yxh_postprocess_ev: once `filter_done` has fired, nothing reads `pred` any more -- a
    forward may overwrite it while the rest of the NMS runs (bench.py's pipelined step)."""
    from yolox_amd.utils.boxes import postprocess_device
    pred = synthetic_pred(3, 2000, 80, 21, dense=True)
    p = torch.from_numpy(pred.copy()).cuda()
    ev, side = torch.cuda.Event(), torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        det, counts = postprocess_device(p, 80, 0.3, 0.65, filter_done=ev)
    torch.cuda.current_stream().wait_event(ev)
    want_xyxy = p[..., :4].clone()  # ordered after the filter's in-place write
    p.fill_(-7.0)  # the next batch's forward
    torch.cuda.synchronize()
    ref = pred.copy()
    want = oracle.postprocess(ref, 80, 0.3, 0.65)
    np.testing.assert_array_equal(want_xyxy.cpu().numpy(), ref[..., :4])
    n = counts.cpu().tolist()
    for b, w in enumerate(want):
        assert n[b] == (0 if w is None else len(w))
        if w is not None:
            np.testing.assert_array_equal(det[b, :n[b]].cpu().numpy(), w)


@pytest.mark.parametrize("empty", [False, True])
def test_split_streams_filter_in_order_rest_beside(oracle, empty):
    """yxh_postprocess_split (bench.py's default serving step): the count reset and the filter on
    the producer's own stream, the sort / mask / reduce on a side stream after `filter_done`.  The
    producer overwrites `pred` right behind the filter in stream order (no event wait) and the
    results stay bit-exact vs the oracle; an all-filtered batch (A > 0, no candidates) too."""
    from yolox_amd.utils.boxes import postprocess_device
    pred = synthetic_pred(3, 2000, 80, 22, dense=True)
    if empty:
        pred[..., 4] = 0.0
    p = torch.from_numpy(pred.copy()).cuda()
    ev, side = torch.cuda.Event(), torch.cuda.Stream()
    det, counts = postprocess_device(p, 80, 0.3, 0.65, filter_done=ev, rest_stream=side)
    want_xyxy = p[..., :4].clone()  # stream order: after the filter's in-place write
    p.fill_(-7.0)  # the next batch's forward, in order on the same stream
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    ref = pred.copy()
    want = oracle.postprocess(ref, 80, 0.3, 0.65)
    np.testing.assert_array_equal(want_xyxy.cpu().numpy(), ref[..., :4])
    n = counts.cpu().tolist()
    for b, w in enumerate(want):
        assert n[b] == (0 if w is None else len(w))
        if w is not None:
            np.testing.assert_array_equal(det[b, :n[b]].cpu().numpy(), w)
    with pytest.raises(ValueError):
        postprocess_device(p, 80, 0.3, 0.65, rest_stream=side)  # the split form needs the event


def test_single_class_many_overlaps(oracle):
    pred = synthetic_pred(2, 1024, 1, 5, dense=True)
    run_both(oracle, pred, 1, 0.0, 0.5)


def test_full_1280_anchor_set_low_conf(oracle):
    """33600 anchors (1280 input) at conf 0.01: > 16384 candidates per image, so the
    score sort runs as LDS chunks + global merge passes (boxes.py:56-67 has no cap)."""
    pred = synthetic_pred(2, 33600, 80, 11)
    pred[..., 4] = np.maximum(pred[..., 4], 0.5)
    pred[..., 5] = np.maximum(pred[..., 5], 0.2)  # every anchor passes conf 0.01
    want = run_both(oracle, pred, 80, 0.01, 0.65)
    assert all(w is not None for w in want)
    run_both(oracle, pred, 80, 0.01, 0.65, agnostic=True)


@pytest.mark.parametrize("A", [16385, 40000])
def test_candidate_counts_past_one_sort_chunk(oracle, A):
    """Candidate counts just past one LDS chunk and past two merge levels, few classes."""
    pred = synthetic_pred(1, A, 3, 13)
    run_both(oracle, pred, 3, 0.0, 0.5)


@pytest.mark.parametrize("budget", [1 << 16, 1 << 20])
def test_mask_passes_match_one_pass(oracle, budget):
    """The suppression matrix in many row passes (tiny mask budget: 64-row passes for the
    first case) gives the oracle's keep lists bit for bit, both batched_nms branches."""
    from yolox_amd import _native as N
    lib = N.lib()
    lib.yxh_set_nms_mask_budget(budget)
    try:
        pred = synthetic_pred(2, 6000, 80, 17)
        pred[..., 4] = np.maximum(pred[..., 4], 0.5)
        run_both(oracle, pred, 80, 0.05, 0.65)
        run_both(oracle, pred, 80, 0.05, 0.65, agnostic=True)
        pred = synthetic_pred(1, 3000, 2, 19, dense=True)
        run_both(oracle, pred, 2, 0.0, 0.5)
    finally:
        lib.yxh_set_nms_mask_budget(0)


@pytest.mark.parametrize("name,dtype,size,batch", [("yolox_s", torch.bfloat16, 320, 4), ("yolox_s", torch.bfloat16, 640, 2),
                                                    ("yolox_l", torch.float16, 320, 2)])  # yolox_l: 256-channel head
def test_scored_filter_from_head_records(oracle, name, dtype, size, batch):
    """Plan.enable_scores (ABI 18): the head launches also write per-anchor records {obj * max class,
    max class, class index, obj, cx, cy, w, h}; (1) the output rows are bit-identical to a plan without records,
    (2) every record equals the filter's own arithmetic on its row (first maximum, obj * conf in fp32),
    (3) yxh_postprocess_scored's detections, counts and in-place xyxy rows are bit-identical to the
    row-reading filter's and to the C oracle's, at three thresholds, on one stream and split over two."""
    from yolox_amd import _native as N
    from yolox_amd.engine import Plan
    from yolox_amd.models import YoloxModule
    from yolox_amd.utils.boxes import postprocess_device
    from yolox_amd.weights import synthetic_images
    m = YoloxModule.synthetic(name, seed=0, device="cuda", dtype=dtype)
    x = torch.from_numpy(synthetic_images(batch, size, size, seed=21)).cuda()
    plain = Plan(m, batch, size, size, dtype, "cuda", N.NHWC, torch.uint8)
    plain.static_input().copy_(x)
    want_rows = plain.replay().clone()
    p = Plan(m, batch, size, size, dtype, "cuda", N.NHWC, torch.uint8)
    scores = p.enable_scores()
    assert scores is not None and tuple(scores.shape) == (batch, p.anchors, 8)
    p.static_input().copy_(x)
    rows = p.replay().clone()
    torch.cuda.synchronize()
    assert torch.equal(rows, want_rows)
    h = rows.cpu().numpy()
    cls = h[..., 5:]
    best = cls.max(-1)
    rec = scores.cpu().numpy()
    np.testing.assert_array_equal(rec[..., 1], best)
    np.testing.assert_array_equal(rec[..., 2], cls.argmax(-1).astype(np.float32))
    np.testing.assert_array_equal(rec[..., 3], h[..., 4])
    np.testing.assert_array_equal(rec[..., 0], (h[..., 4] * best).astype(np.float32))
    np.testing.assert_array_equal(rec[..., 4:8], h[..., :4])  # the row's cxcywh box
    side = torch.cuda.Stream()
    for conf in (0.01, 0.3, 0.5):
        want = oracle.postprocess(h.copy(), 80, conf, 0.65)
        pa, pb = rows.clone(), rows.clone()
        da, ca = postprocess_device(pa, 80, conf, 0.65)
        db, cb = postprocess_device(pb, 80, conf, 0.65, scores=scores)
        ev = torch.cuda.Event()
        pc = rows.clone()
        dc, cc = postprocess_device(pc, 80, conf, 0.65, scores=scores, filter_done=ev, rest_stream=side)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        assert torch.equal(pa, pb) and torch.equal(pa, pc)  # the in-place xyxy rows
        assert torch.equal(ca, cb) and torch.equal(ca, cc)
        n = ca.cpu().numpy()
        for b in range(batch):
            assert torch.equal(da[b, :n[b]], db[b, :n[b]]) and torch.equal(da[b, :n[b]], dc[b, :n[b]])
            if want[b] is None:
                assert n[b] == 0
            else:
                np.testing.assert_array_equal(db[b, :n[b]].cpu().numpy(), want[b])

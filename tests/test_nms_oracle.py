"""Known-answer vectors for the restated torchvision NMS (oracle).

torchvision is absent from the reference checkout and this container, so NMS
parity is pinned by hand-made cases whose answers follow from the published
algorithm (stable descending score order, IoU strictly greater than the threshold,
areas without +1, batched_nms branch rule)."""
import numpy as np
import pytest


def B(*rows):
    return np.array(rows, np.float32).reshape(-1, 4)


def test_basic_suppression_and_order(oracle):
    boxes = B([0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [0, 0, 10, 10.5])
    scores = np.array([0.9, 0.8, 0.7, 0.95], np.float32)
    # box3 (0.95) first; box0 IoU(box3)=100/105>0.5 suppressed; box1 IoU(box3)=
    # 81*... > 0.5? inter=(10-1)*(10.5-1)=85.5, union=105+100-85.5=119.5 -> 0.715 -> suppressed
    keep = oracle.nms(boxes, scores, 0.5)
    assert keep.tolist() == [3, 2]


def test_threshold_is_strict_greater(oracle):
    # IoU exactly 0.5: inter 50, areas 100 and 50 ... choose boxes with IoU = 1/2 exactly
    boxes = B([0, 0, 10, 10], [0, 0, 10, 5])  # inter 50, union 100 -> 0.5
    scores = np.array([0.9, 0.8], np.float32)
    assert oracle.nms(boxes, scores, 0.5).tolist() == [0, 1]
    assert oracle.nms(boxes, scores, 0.4999).tolist() == [0]


def test_no_plus_one_in_area(oracle):
    # with +1 areas (demo_utils.nms) IoU differs; zero-area boxes never suppress
    boxes = B([0, 0, 0, 0], [0, 0, 0, 0])
    scores = np.array([0.5, 0.6], np.float32)
    assert oracle.nms(boxes, scores, 0.1).tolist() == [1, 0]  # 0/0 -> nan, nan > t is False


def test_ties_keep_index_order(oracle):
    boxes = B([0, 0, 1, 1], [10, 10, 11, 11], [20, 20, 21, 21])
    scores = np.array([0.5, 0.5, 0.5], np.float32)
    assert oracle.nms(boxes, scores, 0.5).tolist() == [0, 1, 2]


def test_batched_classes_do_not_interact(oracle):
    boxes = B([0, 0, 10, 10], [0, 0, 10, 10], [0, 0, 10, 10])
    scores = np.array([0.9, 0.8, 0.7], np.float32)
    idxs = np.array([0, 1, 0], np.float32)
    # trick branch (numel 12 <= 4000) and vanilla branch (limit 0) agree here
    assert oracle.batched_nms(boxes, scores, idxs, 0.5).tolist() == [0, 1]
    assert oracle.batched_nms(boxes, scores, idxs, 0.5, vanilla_numel=0).tolist() == [0, 1]


def test_coordinate_trick_can_merge_classes_with_negative_coords(oracle):
    """The offset trick assumes coordinates >= 0: with a large negative x1 a box of
    class 1 can overlap a class-0 box after shifting, so the trick branch suppresses
    across classes while the vanilla branch does not -- both restated faithfully."""
    boxes = B([0, 0, 10, 10], [-11, -11, -1, -1])  # max coord 10 -> class-1 offset 11 -> [0,0,10,10]
    scores = np.array([0.9, 0.8], np.float32)
    idxs = np.array([0, 1], np.float32)
    assert oracle.batched_nms(boxes, scores, idxs, 0.5).tolist() == [0]
    assert oracle.batched_nms(boxes, scores, idxs, 0.5, vanilla_numel=0).tolist() == [0, 1]


def test_postprocess_none_and_inplace(oracle):
    pred = np.zeros((2, 3, 5 + 2), np.float32)
    pred[0, 0, :4] = [10, 10, 4, 6]
    pred[0, 0, 4] = 0.9
    pred[0, 0, 5:] = [0.2, 0.8]
    out = oracle.postprocess(pred, 2, 0.5, 0.45)
    assert out[1] is None
    assert out[0].shape == (1, 7)
    np.testing.assert_array_equal(out[0][0], np.array([8, 7, 12, 13, 0.9, 0.8, 1], np.float32))
    np.testing.assert_array_equal(pred[0, 0, :4], [8, 7, 12, 13])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_greedy_equals_bruteforce_definition(oracle, seed):
    """Cross-check the C restatement against a direct numpy statement of greedy NMS."""
    rng = np.random.default_rng(seed)
    xy = rng.uniform(0, 100, (300, 2)).astype(np.float32)
    wh = rng.uniform(5, 40, (300, 2)).astype(np.float32)
    boxes = np.concatenate([xy, xy + wh], 1).astype(np.float32)
    scores = rng.uniform(0, 1, 300).astype(np.float32)
    order = sorted(range(300), key=lambda i: (-scores[i], i))
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    keep, removed = [], np.zeros(300, bool)
    for i in order:
        if removed[i]:
            continue
        keep.append(i)
        for j in order:
            if removed[j] or j == i:
                continue
            xx1 = max(boxes[i, 0], boxes[j, 0]); yy1 = max(boxes[i, 1], boxes[j, 1])
            xx2 = min(boxes[i, 2], boxes[j, 2]); yy2 = min(boxes[i, 3], boxes[j, 3])
            w = np.float32(max(np.float32(0), np.float32(xx2 - xx1)))
            h = np.float32(max(np.float32(0), np.float32(yy2 - yy1)))
            inter = np.float32(w * h)
            ovr = np.float32(inter / np.float32(np.float32(area[i] + area[j]) - inter))
            if float(ovr) > 0.45 and order.index(j) > order.index(i):
                removed[j] = True
    assert oracle.nms(boxes, scores, 0.45).tolist() == keep

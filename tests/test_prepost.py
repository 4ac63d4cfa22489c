"""Pre/post-processing rows: letterbox geometry, cv2-INTER_LINEAR restatement, u8
normalisation, scale_boxes — CPU checks against the reference's fixtures (prepost.npz) and GPU parity of
the HIP kernels (fce_letterbox / fce_scale_boxes / u8 stem input) against the oracle."""

import ctypes as C

import numpy as np
import pytest
import torch

import cases
from fce_yolo_amd import _native as N
from fce_yolo_amd import predict as P
from fce_yolo_amd.engine import Engine
from oracle import nms_oracle
from oracle import preprocess_oracle as PO


@pytest.fixture(scope="module")
def pp():
    from conftest import GOLDEN

    return np.load(GOLDEN / "prepost.npz", allow_pickle=False)


def test_oracle_letterbox_geometry_matches_reference(pp):
    for H, W, h0, w0, new_h, new_w, top, bottom, left, right, value in pp["geometry"]:
        assert PO.letterbox_geometry(h0, w0, H, W) == (new_h, new_w, top, bottom, left, right)
        assert top + new_h + bottom == H and left + new_w + right == W and value == 114


def test_product_letterbox_geometry_matches_reference(pp):
    for H, W, h0, w0, new_h, new_w, top, _, left, _, _ in pp["geometry"]:
        assert P.letterbox_geometry(int(h0), int(w0), int(H), int(W)) == (new_h, new_w, top, left)


def test_oracle_scale_boxes_matches_reference(pp):
    for i, (H, W, h0, w0) in enumerate(pp["sb_cases"]):
        got = PO.scale_boxes((H, W), pp[f"sb{i}/boxes"], (h0, w0, 3))
        assert np.array_equal(got, pp[f"sb{i}/out"]), i


def test_product_box_scale_params(pp):
    for H, W, h0, w0 in pp["sb_cases"]:
        gain, px, py = P.box_scale(int(H), int(W), int(h0), int(w0))
        assert gain == min(H / h0, W / w0)
        assert (px, py) == (round((W - w0 * gain) / 2 - 0.1), round((H - h0 * gain) / 2 - 0.1))


def test_resize_restatement_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(PO.resize_linear_u8(img, 53, 37), img)  # no resize: exact copy (fixture-covered)
    const = np.full((40, 60, 3), 77, np.uint8)
    for nw, nh in ((123, 81), (17, 11), (60, 41)):
        assert (PO.resize_linear_u8(const, nw, nh) == 77).all()  # coefficients sum to 2048 -> exact


def test_letterbox_structs_match_header():
    assert C.sizeof(P.LetterboxImg) == 8 + 7 * 4 + 4  # pointer + 7 ints, padded to 8
    assert C.sizeof(P.BoxScale) == 20


# ------------------------------------------------------------------------------------------------ GPU


def _images(rng, shapes):
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]


@pytest.mark.gpu
def test_letterbox_kernel_bit_exact_vs_oracle(device):
    rng = np.random.default_rng(1)
    shapes = [(480, 640), (640, 480), (333, 517), (100, 100), (17, 999), (640, 640), (1080, 1920), (5, 6)]
    imgs = _images(rng, shapes)
    for H, W in ((640, 640), (320, 320), (384, 640)):
        lb = P.Letterbox(len(imgs), (H, W), device)
        out = lb([torch.from_numpy(im).to(device) for im in imgs]).cpu().numpy()
        ref, _ = PO.preprocess(imgs, H, W)
        for i in range(len(imgs)):
            assert np.array_equal(out[i], ref[i]), (H, W, shapes[i])


@pytest.mark.gpu
def test_scale_boxes_kernel_bit_exact_vs_reference(pp, device):
    cs = pp["sb_cases"]
    n, md = len(cs), 64
    dets = torch.zeros(n, md, 6)
    host = (P.BoxScale * n)()
    for i, (H, W, h0, w0) in enumerate(cs):
        dets[i, :, :4] = torch.from_numpy(pp[f"sb{i}/boxes"])
        gain, px, py = P.box_scale(int(H), int(W), int(h0), int(w0))
        host[i] = P.BoxScale(gain, px, py, int(h0), int(w0))
    counts = torch.full((n,), md, dtype=torch.int32, device=device)
    counts[3] = 10  # slots past the count stay untouched
    d = dets.to(device)
    sc = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8).to(device)
    N.call("fce_scale_boxes", C.c_void_p(d.data_ptr()), C.c_void_p(counts.data_ptr()), n, md,
           C.c_void_p(sc.data_ptr()), None)
    d = d.cpu()
    for i in range(n):
        k = int(counts[i])
        assert np.array_equal(d[i, :k, :4].numpy(), pp[f"sb{i}/out"][:k]), i
        assert torch.equal(d[i, k:], dets[i, k:]), i


@pytest.mark.gpu
def test_u8_input_matches_half_div_255(device):
    """Engine fed the u8 canvas == engine fed the reference's `im.half() / 255` tensor (bitwise)."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    rng = np.random.default_rng(2)
    x8 = torch.from_numpy(rng.integers(0, 256, (2, 3, 160, 160), dtype=np.uint8))
    eng = Engine(model, 2, 160, device)
    a = eng(x8.to(device)).clone()
    b = eng((x8.half() / 255).to(device)).clone()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_predictor_end_to_end_vs_oracle(device):
    """Mixed-size uint8 images -> device letterbox -> forward -> NMS -> scale_boxes, against the oracle
    chain (letterbox restatement, oracle fp32 forward, oracle NMS, reference scale_boxes) on a model whose
    boxes are compared within the forward tolerance and whose NMS is checked on our own predictions."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    rng = np.random.default_rng(3)
    shapes = [(240, 320), (320, 200), (150, 150)]
    imgs = _images(rng, shapes)
    pred = P.Predictor(model, 4, 320, device)
    dets, keep = pred(imgs, return_idxs=True)
    assert len(dets) == 3
    # oracle chain on our own forward output (forward parity is covered by the e2e tests)
    canvas = torch.from_numpy(PO.preprocess(imgs, 320, 320)[0])
    full = torch.cat([canvas, canvas[-1:]], 0).to(device)
    y = pred.engine(full).clone().cpu().numpy()
    od, ok = nms_oracle.non_max_suppression(y)
    for i, (h0, w0) in enumerate(shapes):
        assert np.array_equal(keep[i].cpu().numpy(), ok[i])
        ref = PO.scale_boxes((320, 320), od[i][:, :4], (h0, w0, 3))
        got = dets[i].cpu().numpy()
        assert np.array_equal(got[:, :4], ref) and np.array_equal(got[:, 4:], od[i][:, 4:])
    pred.close()


@pytest.mark.gpu
def test_predictor_stream_matches_one_at_a_time(device):
    """The overlapped predictor (3 slots in flight: pinned staging, one H2D / D2H copy per batch, hipGraph
    lanes) gives every batch exactly what a one-lane, direct-launch predictor gives it; partial batches,
    more batches than slots, and results collected out of order after their slots were reused."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    rng = np.random.default_rng(4)
    batches = [_images(rng, [(240, 320), (320, 200), (150, 150), (480, 640)]), _images(rng, [(100, 333)]),
               _images(rng, [(320, 320)] * 4), _images(rng, [(64, 512), (512, 64), (300, 301)]),
               _images(rng, [(200, 180)] * 4)]
    p1 = P.Predictor(model, 4, 320, device, lanes=1, graph=False)
    seq = [p1(b, return_idxs=True) for b in batches]
    p1.close()
    p3 = P.Predictor(model, 4, 320, device, lanes=3)

    def same(a, b):
        return len(a[0]) == len(b[0]) and all(torch.equal(x, y) for x, y in zip(a[0] + a[1], b[0] + b[1]))

    for i, r in enumerate(p3.stream(batches, return_idxs=True)):
        assert same(r, seq[i]), i
    tickets = [p3.submit(b) for b in batches]  # 5 batches over 3 slots: two collected early
    for i in reversed(range(len(batches))):
        assert same(p3.result(tickets[i], return_idxs=True), seq[i]), i
    with pytest.raises(KeyError):
        p3.result(tickets[0])
    p3.close()

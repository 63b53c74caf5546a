"""Weight plumbing: reference key sets, VDW1 round trip, synthetic inputs."""
import numpy as np
import torch

from oracle.retinaface import RetinaFaceMnet, RetinaFaceR50, build_oracle_model


def test_retinaface_keys_match_reference_module_tree():
    from vdmi import weights
    sd = weights.retinaface_state_dict(0)
    ref = {k: tuple(v.shape) for k, v in RetinaFaceR50().state_dict().items()
           if not k.endswith("num_batches_tracked")}
    assert set(sd) == set(ref)
    for k, v in sd.items():
        assert v.shape == ref[k], k
    # spot-check reference names (retinaface.py:73-92, layers.py:44-52,72-77)
    for k in ("body.conv1.weight", "body.layer1.0.conv1.weight", "body.layer2.0.downsample.0.weight",
              "fpn.output1.0.weight", "fpn.merge2.1.running_var", "ssh1.conv3X3.0.weight",
              "ssh3.conv7x7_3.1.bias", "ClassHead.0.conv1x1.weight", "LandmarkHead.2.conv1x1.bias"):
        assert k in sd
    assert sum(v.size for k, v in sd.items() if k.endswith("weight") and v.ndim == 4) > 27e6


def test_retinaface_mnet_keys_match_reference_module_tree():
    """backbone="mobilenet": MobileNetV1 stage1..3 (mobilenet025.py:21-48) + FPN/SSH/heads at 64."""
    from vdmi import weights
    sd = weights.retinaface_mnet_state_dict(0)
    ref = {k: tuple(v.shape) for k, v in RetinaFaceMnet().state_dict().items()
           if not k.endswith("num_batches_tracked")}
    assert set(sd) == set(ref)
    for k, v in sd.items():
        assert v.shape == ref[k], k
    for k, shape in (("body.stage1.0.0.weight", (8, 3, 3, 3)), ("body.stage1.1.0.weight", (8, 1, 3, 3)),
                     ("body.stage1.5.4.running_var", (64,)), ("body.stage2.0.3.weight", (128, 64, 1, 1)),
                     ("body.stage3.1.3.weight", (256, 256, 1, 1)), ("fpn.output3.0.weight", (64, 256, 1, 1)),
                     ("ssh1.conv5X5_1.0.weight", (16, 64, 3, 3)), ("ClassHead.2.conv1x1.weight", (4, 64, 1, 1))):
        assert sd[k].shape == shape, k
    m = build_oracle_model(sd)
    assert isinstance(m, RetinaFaceMnet)
    with torch.no_grad():
        loc, conf, _ = m(torch.zeros(1, 3, 64, 64))
    assert loc.shape == (1, 168, 4) and torch.allclose(conf.sum(-1), torch.ones(1, 168))


def test_weights_deterministic_and_vdw_roundtrip():
    from vdmi import weights
    a = weights.retinaface_state_dict(0)
    b = weights.retinaface_state_dict(0)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    blob = weights.pack_vdw(a)
    assert blob[:4] == b"VDW1"
    back = weights.unpack_vdw(blob)
    assert set(back) == set(a) and all(np.array_equal(back[k], a[k]) for k in a)
    # integer buffers are skipped
    assert "x" not in weights.unpack_vdw(weights.pack_vdw({"x": np.arange(3), "y": np.ones(2, np.float32)}))


def test_oracle_model_runs_small():
    from vdmi import weights
    m = build_oracle_model(weights.retinaface_state_dict(0))
    with torch.no_grad():
        loc, conf, ldm = m(torch.zeros(1, 3, 64, 64))
    assert loc.shape == (1, 2 * (64 + 16 + 4), 4) and conf.shape[-1] == 2 and ldm.shape[-1] == 10
    assert torch.allclose(conf.sum(-1), torch.ones(1, 168))


def test_synthetic_frames_deterministic():
    from vdmi import synth
    f1 = synth.frames(2, 16, 24, seed=0)
    f2 = synth.frames(2, 16, 24, seed=0)
    assert f1.dtype == np.uint8 and np.array_equal(f1, f2)
    assert not np.array_equal(f1[0], f1[1])
    assert not np.array_equal(synth.frame(16, 24, 0, seed=1), f1[0])
    b = synth.box_lists(4, 1080, 1920)
    assert b.shape == (4, 8, 4) and (b[..., 2] > b[..., 0]).all()


def test_yolov8n_keys_match_ultralytics_tree():
    from oracle.yolov8 import YOLOv8n
    from vdmi import weights
    sd = weights.yolov8n_state_dict(0, nc=1)
    ref = {k: tuple(v.shape) for k, v in YOLOv8n(1).state_dict().items() if not k.endswith("num_batches_tracked")}
    assert set(sd) == set(ref), set(sd) ^ set(ref)
    for k, v in sd.items():
        assert v.shape == ref[k], k
    n = sum(v.size for k, v in sd.items())
    assert 2.9e6 < n < 3.3e6          # YOLOv8n ~3.0-3.2 M parameters


def test_oracle_yolo_runs_small():
    from oracle.yolov8 import build_oracle_yolo, postprocess, raw_heads
    from vdmi import weights
    m = build_oracle_yolo(weights.yolov8n_state_dict(0))
    with torch.no_grad():
        lv = m(torch.zeros(1, 3, 64, 96))
    assert [tuple(t.shape) for t in lv] == [(1, 65, 8, 12), (1, 65, 4, 6), (1, 65, 2, 3)]
    raw = raw_heads(lv)
    res = postprocess(raw, [(8, 12), (4, 6), (2, 3)], (64, 96), (64, 96))
    assert len(res) == 1


def test_dropins_refuse_missing_weights():
    """A missing checkpoint is an error, never a silent switch to random weights
    (a desensitisation run on random weights leaves faces visible)."""
    import pytest as _pt
    from vdmi import plate
    with _pt.raises(FileNotFoundError):
        plate.load_plate_weights("/nonexistent/best.pt")


def test_plate_weights_refuse_pickled_objects(tmp_path):
    """A pickled ultralytics-style object is refused by the weights-only loader; a
    converted state_dict file loads."""
    import fractions

    import pytest as _pt
    import torch
    from vdmi import plate, weights

    bad = tmp_path / "best.pt"     # an arbitrary pickled object stands in for an ultralytics model
    torch.save({"model": fractions.Fraction(1, 3)}, bad)
    with _pt.raises(ValueError):
        plate.load_plate_weights(str(bad))
    sd = {k: torch.from_numpy(v) for k, v in weights.yolov8n_state_dict(0).items()}
    good = tmp_path / "best_sd.pt"
    torch.save(sd, good)
    got = plate.load_plate_weights(str(good))
    assert set(got) == set(sd) and all(np.array_equal(got[k], sd[k].numpy()) for k in sd)

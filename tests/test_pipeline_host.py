"""batch_process_images host-side semantics that need no GPU (combine_detect.py:183-277)."""
import os

import pytest


def test_gpu_codec_with_custom_io_is_refused(tmp_path):
    """gpu_codec=True reads/writes JPEG bytes itself; a caller's loader/saver would be
    silently ignored, so the combination is an error."""
    from vdmi.pipeline import batch_process_images
    with pytest.raises(ValueError, match="custom loader"):
        batch_process_images(str(tmp_path), str(tmp_path / "o"), object(), object(), gpu_codec=True,
                             loader=lambda p: None)


def test_load_failure_aborts_generic_detectors(tmp_path):
    """Generic detector objects take the reference's two-thread path; a loader error
    propagates out of the call (combine_detect.py:209-211: outside the try)."""
    from vdmi.pipeline import batch_process_images
    (tmp_path / "a.jpg").write_bytes(b"")

    def loader(p):
        raise ValueError(f"cannot read image: {p}")

    calls = []
    with pytest.raises(ValueError, match="cannot read"):
        batch_process_images(str(tmp_path), str(tmp_path / "o"), object(), lambda *a, **k: calls.append(1),
                             loader=loader, saver=lambda *a: None)
    assert not calls and os.path.isdir(tmp_path / "o")

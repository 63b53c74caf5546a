import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "video-desensitization_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvdmi.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "parity: oracle box-parity test (ordered first in the session)")


def pytest_collection_modifyitems(session, config, items):
    """Oracle parity tests run first, so a later -x stop cannot hide them."""
    items.sort(key=lambda it: 0 if it.get_closest_marker("parity") else 1)


def _have_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _have_gpu():
        pytest.skip("no GPU")
    import vdmi
    vdmi.load()
    return True


_CTX = {}


@pytest.fixture(scope="session")
def face_ctx_factory(gpu):
    """Cached contexts keyed by (precision, max_batch, weight-kind)."""
    import vdmi
    from vdmi import weights

    def make(precision="fp32", max_batch=8, wkind="default", options=(), **kw):
        key = (precision, max_batch, wkind, tuple(options), tuple(sorted(kw.items())))
        if key not in _CTX:
            ctx = vdmi.Context(precision=precision, max_batch=max_batch, options=dict(options), **kw)
            ctx.load_weights(0, face_weights(wkind))
            _CTX[key] = ctx
        return _CTX[key]

    yield make
    for c in _CTX.values():
        c.close()
    _CTX.clear()


_W = {}


def face_weights(kind="default"):
    from vdmi import weights
    if kind not in _W:
        if kind == "default":
            _W[kind] = weights.retinaface_state_dict(0)
        elif kind == "dense":      # thousands of candidates per frame: stresses sort/NMS paths
            _W[kind] = weights.retinaface_state_dict(0, cls_bias={0: -2.0, 1: -1.0, 2: 0.5})
        elif kind == "mnet":       # backbone="mobilenet" (cfg_mnet)
            _W[kind] = weights.retinaface_mnet_state_dict(0)
        else:
            raise KeyError(kind)
    return _W[kind]

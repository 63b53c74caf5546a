"""CPU-side checks of the C-ABI boundary: libvdmi.so loads, exports every entry
point include/vdmi.h declares, and its host-only calls behave (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _header_functions():
    src = open(os.path.join(ROOT, "include", "vdmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vdt?_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    import vdmi
    from vdmi import _lib
    lib = vdmi.load()
    names = _header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"libvdmi.so does not export {n}"
    bound = {s[0] for s in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirrors of vd_cfg / vd_boxes have the C compiler's size and field offsets."""
    import shutil
    import subprocess
    from vdmi import _lib
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    fields = {"vd_cfg": [f[0] for f in _lib.vd_cfg._fields_], "vd_boxes": [f[0] for f in _lib.vd_boxes._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "vdmi.h"', "int main(void){"]
    for st, fl in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fl:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for st, cls in (("vd_cfg", _lib.vd_cfg), ("vd_boxes", _lib.vd_boxes)):
        assert int(out[st]) == ctypes.sizeof(cls)
        for f in fields[st]:
            assert int(out[f"{st}.{f}"]) == getattr(cls, f).offset, f


def test_default_cfg_and_version():
    from vdmi import _lib
    lib = _lib.load()
    assert lib.vd_abi_version() == 2
    c = _lib.default_cfg()
    assert (c.input_h, c.input_w, c.max_batch) == (640, 640, 64)          # combine_detect.py:860, config.ini:35
    assert abs(c.confidence - 0.5) < 1e-9 and c.nms_iou == 0.4 and c.mosaic_level == 8


def test_errors_are_reported_not_raised_through_abi():
    from vdmi import _lib
    lib = _lib.load()
    assert lib.vd_create(None, 0, None) == _lib.VD_ERR_ARG
    assert "null" in _lib.last_error()
    assert lib.vd_detect(None, None, 0, 0, 0, 0, 0, None) == _lib.VD_ERR_ARG
    assert lib.vd_destroy(None) == _lib.VD_OK


def test_check_raises_typed_errors():
    from vdmi import _lib
    with pytest.raises(_lib.VdCapacityError):
        _lib.check(_lib.VD_ERR_CAPACITY)
    with pytest.raises(_lib.VdError):
        _lib.check(_lib.VD_ERR_ARG)


def test_host_boxes_struct():
    from vdmi import _lib
    hb = _lib.HostBoxes(3, 5)
    s = hb.struct()
    assert s.cap == 5 and s.where == _lib.VD_HOST and s.count == hb.count.ctypes.data
    hb.count[:] = [2, 0, 9]
    assert hb.frame(0)[0].shape == (2, 4) and hb.frame(2)[0].shape == (5, 4)

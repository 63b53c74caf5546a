"""`.record` container I/O for the camera topics: the reference's `recordDeal`
module surface (foreign/recordDeal.so, called at combine_detect.py:839 and :958),
rebuilt as host C++ behind the C-ABI (csrc/record.cpp; vd_record_extract_h265 /
vd_record_repack_h265 in include/vdmi.h).

    read_record2h265_all(record_dir, output_h265_dir)
        every *.record* segment of record_dir -> output_h265_dir/hevcs/<camera>.h265
        (the CompressedImage data of /drivers/camera/<camera>/compressed/image from
        its first key frame on); returns the number of camera streams written.
    write_allH265_record_all(record_dir, videos_dir, record_output_dir)
        the same segments rewritten into record_output_dir with the extracted
        messages' data replaced by the access units of the desensitised stream
        videos_dir/<camera>_processed.h265 (or .hevc, or processed_<camera>.h265;
        the name combine_detect.py:658 gives it); the extract step's un-suffixed
        <camera>.h265 holds the ORIGINAL frames and is refused. Returns the number
        of record files written.

Errors (missing directory, not a CyberRT record, a compressed record) raise
VdError, as the reference's RecordException surfaces them. Only uncompressed
records are handled (no bz2 / lz4 codecs in this image)."""
import ctypes
import os

from . import _lib


def read_record2h265_all(record_dir, output_h265_dir):
    lib = _lib.load()
    n = ctypes.c_int(0)
    _lib.check(lib.vd_record_extract_h265(os.fsencode(record_dir), os.fsencode(output_h265_dir), ctypes.byref(n)))
    return n.value


def write_allH265_record_all(record_dir, videos_dir, record_output_dir):
    lib = _lib.load()
    n = ctypes.c_int(0)
    _lib.check(lib.vd_record_repack_h265(os.fsencode(record_dir), os.fsencode(videos_dir),
                                         os.fsencode(record_output_dir), ctypes.byref(n)))
    return n.value

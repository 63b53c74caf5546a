"""Build libvdmi.so (HIP, gfx950), in-tree.

    python video-desensitization_amd/build.py            # incremental
    python video-desensitization_amd/build.py --force    # rebuild everything

Each translation unit is compiled to an object under build/ (skipped when the
object is newer than its sources and headers), then linked into
video-desensitization_amd/vdmi/libvdmi.so, next to the Python package that
loads it. No CMake, no torch extension machinery: plain hipcc.
"""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "vdmi", "libvdmi.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("VD_OFFLOAD_ARCH", "gfx950")

SOURCES = ["conv.hip", "conv1x1.hip", "conv_big.hip", "pre.hip", "post.hip", "mosaic.hip", "block.hip", "block32.hip", "block.cpp",
           "chain.hip", "chain32.hip", "stem.hip", "dwconv.hip", "conv_x6.hip", "jpeg.hip", "jpeg_dec.hip", "jpeg_host.cpp", "jpeg_enc.hip", "jpeg_enc.cpp", "runtime.cpp", "face_net.cpp", "plate_net.cpp", "record.cpp"]
HEADERS = ["vd_common.h", "vd_math.h", "nets.h"]
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", f"-I{os.path.join(ROOT, 'include')}"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src, force):
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "vdmi.h")]
    if not force and not _newer(o, deps):
        return o, None
    lang = ["-x", "hip"]
    cmd = [HIPCC] + FLAGS + lang + ["-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return o, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return o, None


def build(force=False, jobs=8):
    os.makedirs(OBJ, exist_ok=True)
    missing = [s for s in SOURCES if not os.path.exists(os.path.join(CSRC, s))]
    if missing:
        raise FileNotFoundError(f"missing sources: {missing}")
    srcs = SOURCES
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or _newer(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    args = ap.parse_args()
    lib = build(args.force, args.j)
    print(lib)


if __name__ == "__main__":
    sys.exit(main())

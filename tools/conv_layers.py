"""Per-layer view of a rocprofv3 kernel trace of bench.py: maps the conv launches
of the last step onto the RetinaFace plan (same order as face_net.cpp) and
prints duration and achieved TFLOP/s per layer.

    python tools/conv_layers.py gpurun_out/prof/run_kernel_trace.csv [batch]
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import face_stream  # noqa: E402


def face_plan(B=64, H=640, W=640, fused=True, block=True, chain=True, ssh_fused=True, dual=(0, 1)):
    """(name, M, N, K) of every conv launch in face_net.cpp order; with `block` the
    three layer1 bottlenecks are one launch each (block.hip), K = their summed
    reduction depth per output channel of 256 (same FLOPs); with `chain`
    layer2.1/2.2's conv3 runs with the next block's conv1 (chain.hip, N=512 K=256
    carries both layers' FLOPs; a tuple names the layer2 blocks bi whose conv3 chains with
    block bi+1's conv1, a dict {layer index: blocks} any layer's: the fp32 plan's chain32.hip
    takes {1: (0, 1, 2), 2: (0, 1, 2, 3, 4)}); with `ssh_fused` each SSH's conv5X5_1 and conv3X3
    are one 192-channel conv; `dual`: the layers whose block 0 runs conv3 + downsample
    as one launch (bf16: layer1/2; fp32: layer1)."""
    L = []
    if isinstance(chain, dict):          # {layer index: blocks whose conv3 chains with the next conv1}
        chained = {li: tuple(v) for li, v in chain.items()}
    else:
        chained = {1: tuple(chain) if isinstance(chain, (tuple, list)) else ((1, 2) if chain else ())}
    h, w = H // 2, W // 2
    L.append(("stem7x7", B * h * w, 64, 3 * 49))
    h, w = h // 2, w // 2
    cin = 64
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for bi in range(blocks):
            s = stride if bi == 0 else 1
            if block and li == 0:
                k = (cin * 64 + 576 * 64 + 64 * 256 + (cin * 256 if bi == 0 else 0)) // 256
                L.append((f"l1.{bi}.block", B * h * w, 256, k))
                cin = planes * 4
                continue
            if bi - 1 in chained.get(li, ()):
                pass                            # ran inside the previous block's chain launch
            else:
                L.append((f"l{li+1}.{bi}.c1", B * h * w, planes, cin))
            oh, ow = h // s, w // s
            L.append((f"l{li+1}.{bi}.c2", B * oh * ow, planes, planes * 9))
            if bi == 0 and fused and li in dual:  # conv3 + downsample in one pass
                L.append((f"l{li+1}.{bi}.c3+ds", B * oh * ow, planes * 4, planes + cin))
            else:
                if bi == 0:
                    L.append((f"l{li+1}.{bi}.ds", B * oh * ow, planes * 4, cin))
                if bi in chained.get(li, ()):
                    L.append((f"l{li+1}.{bi}.c3+c1", B * oh * ow, planes * 4, 2 * planes))
                else:
                    L.append((f"l{li+1}.{bi}.c3", B * oh * ow, planes * 4, planes))
            cin = planes * 4
            h, w = oh, ow
    s = [(H // 8, 512), (H // 16, 1024), (H // 32, 2048)]
    L.append(("fpn.o3", B * s[2][0] ** 2, 256, 2048))
    L.append(("fpn.o2", B * s[1][0] ** 2, 256, 1024))
    L.append(("fpn.m2", B * s[1][0] ** 2, 256, 256 * 9))
    L.append(("fpn.o1", B * s[0][0] ** 2, 256, 512))
    L.append(("fpn.m1", B * s[0][0] ** 2, 256, 256 * 9))
    for l, hh in enumerate((H // 8, H // 16, H // 32)):
        m = B * hh * hh
        L += ([(f"ssh{l}.c51+c3", m, 192, 2304)] if ssh_fused else
              [(f"ssh{l}.c3", m, 128, 2304), (f"ssh{l}.c51", m, 64, 2304)])
        if ssh_fused == 2:   # conv5X5_2 + conv7X7_2 as one conv too (option ssh_fuse=2)
            L += [(f"ssh{l}.c52+c72", m, 128, 576), (f"ssh{l}.c73", m, 64, 576), (f"head{l}", m, 32, 256)]
        else:
            L += [(f"ssh{l}.c52", m, 64, 576),
                  (f"ssh{l}.c72", m, 64, 576), (f"ssh{l}.c73", m, 64, 576), (f"head{l}", m, 32, 256)]
    return L


def main(path, B=64):
    allk = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    plan = face_plan(B)
    # The face forward may share the GPU with the plate network on a second
    # stream: anchor on the last face letterbox (space-to-depth form in bf16)
    # and take the conv launches that follow it on the same stream.
    conv_keys = ("conv_igemm", "conv1x1_stream", "conv_big", "bottleneck_kernel", "stem_pool_kernel", "chain_kernel",
                 "conv_persist")
    plan = face_plan(B, block=any("bottleneck_kernel" in r["Kernel_Name"] for r in allk),
                     chain=any("chain_kernel" in r["Kernel_Name"] for r in allk))
    face = face_stream(allk)
    li = max(i for i, r in enumerate(allk) if r["Stream_Id"] in face and "letterbox" in r["Kernel_Name"])
    stream = allk[li]["Stream_Id"]
    last = [r for r in allk[li:] if r["Stream_Id"] == stream and any(k in r["Kernel_Name"] for k in conv_keys)]
    last = last[:len(plan)]
    tot_t = tot_f = 0
    for (name, M, N, K), r in zip(plan, last):
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        fl = 2.0 * M * N * K
        tot_t += dt
        tot_f += fl
        n_ = r["Kernel_Name"]
        kn = ("STEM+POOL" if "stem_pool" in n_ else "BLOCK" if "bottleneck" in n_ else "BIG" if "conv_big" in n_
              else "CHAIN" if "chain_kernel" in n_ else "S:" + n_.split("<")[1][:12] if "conv1x1_stream" in n_
              else "G:" + n_.split("conv_igemm_kernel")[1][:22] if "conv_igemm_kernel" in n_ else n_[:24])
        print(f"{name:12s} M={M:8d} N={N:5d} K={K:5d} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s  {kn}")
    print(f"total {tot_t*1e3:.2f} ms  {tot_f/tot_t/1e12:.1f} TF/s")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64)

"""Chunk timeline of the x3 NT ring (debug-ablation build, KAIR_LIB=debug KAIR_RING_DBG=8): one launch of a
micro-benchmark case, then per CTA 0..3 the mean cycles per iteration spent in each phase (waiting for the
chunk, barrier + DMA issue, MFMAs, epilogue) and the spread of the loop-top times over the 8 waves.

    KAIR_LIB=debug KAIR_RING_DBG=8 python tools/x3_stamps.py [case]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from tools import x3_micro  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "nt_qkv_fwd"
    run = x3_micro.cases()[name][0]
    run()
    torch.cuda.synchronize()
    H.debug_x3_stamps()   # clear
    run()
    torch.cuda.synchronize()
    st = H.debug_x3_stamps().astype(np.int64).reshape(4, 8, 64, 5)
    print(name)
    for c in range(4):
        s = st[c]
        ok = (s[:, :, 0] > 0).all(axis=0)
        n = int(ok.sum())
        if n < 2:
            continue
        s = s[:, :n]
        d = np.diff(s, axis=2).mean(axis=(0, 1))
        it = np.diff(s[:, :, 0], axis=1).mean()
        spread = (s[:, :, 0].max(axis=0) - s[:, :, 0].min(axis=0)).mean()
        print(f"CTA {c}: {n} iterations, {it:7.0f} cycles/iteration; wait {d[0]:6.0f}  barrier+issue {d[1]:6.0f}  "
              f"mfma {d[2]:6.0f}  epilogue {d[3]:6.0f}; wave skew at loop top {spread:6.0f}")
        ep = s[:, :, 4] - s[:, :, 3]
        big = np.argsort(-ep.mean(axis=0))[:3]
        print("   longest epilogue iterations:", [(int(i), int(ep[:, i].mean())) for i in big],
              " wait per iteration (wave 0):", (s[0, :16, 1] - s[0, :16, 0]).tolist())


if __name__ == "__main__":
    main()

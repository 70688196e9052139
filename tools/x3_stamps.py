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
        for g, (p1, p2) in enumerate((("frags", "mfma+epi"), ("mfma+epi", "frags"))):
            s = st[c, 4 * g:4 * g + 4]
            ok = (s > 0).all(axis=(0, 2))   # intervals every wave of the group stamped at every point
            idx = np.nonzero(ok)[0]
            if len(idx) < 3:
                continue
            s = s[:, idx]
            d = np.diff(s, axis=2).mean(axis=(0, 1))
            it = np.diff(s[:, :, 0], axis=1).mean()
            skew = (st[c, :, idx, 0].max(axis=1) - st[c, :, idx, 0].min(axis=1)).mean()
            ph2 = s[:, :, 4] - s[:, :, 3]
            print(f"CTA {c} group {g}: {len(idx)} intervals, {it:6.0f} cycles/interval; wait {d[0]:5.0f}  barrier+DMA "
                  f"{d[1]:5.0f}  {p1} {d[2]:5.0f}  {p2} {d[3]:5.0f}  (max {ph2.mean(axis=0).max():5.0f}); skew {skew:5.0f}")


if __name__ == "__main__":
    main()

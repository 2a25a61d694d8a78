"""Tail model of the two neighbour passes from the workgroup timelines of scripts/block_times.py
(gpurun_out/block_times_<state>.npy, a -DSPH_BTIME library): list scheduling of the measured workgroup durations onto
each XCD's resident slots (blockIdx b runs on XCD b % 8, in dispatch order), checked against the measured span, then
the same durations dealt heaviest-first per XCD (an ideal longest-processing-time order, known in advance) and over
the whole chip. The LPT spans bound what a cost-ordered tile mapping could buy; it ignores the L2 locality the
XCD-run mapping (common.h xcd_block) keeps."""
import heapq
import sys
from pathlib import Path

import numpy as np

SLOTS_PER_CU = {"density": 7, "force": 4}
CUS_PER_XCD, NX = 32, 8


def span(durs, slots):
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for d in durs:
        t = heapq.heappop(free) + d
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
    for state in ("rest", "mid-collapse"):
        t = np.load(root / f"block_times_{state}.npy")
        for k, name in enumerate(("density", "force")):
            st, en = t[k, :, 0], t[k, :, 1]
            dur = en - st
            meas = en.max() - st.min()
            per = SLOTS_PER_CU[name] * CUS_PER_XCD
            xcd = [dur[x::NX] for x in range(NX)]
            disp = max(span(d, per) for d in xcd)
            lpt_x = max(span(np.sort(d)[::-1], per) for d in xcd)
            lpt_all = span(np.sort(dur)[::-1], per * NX)
            filled = dur.sum() / (per * NX)
            print(f"{state:13s} {name:8s} measured {meas:6.1f} us | model, dispatch order {disp:6.1f} | heaviest first "
                  f"per XCD {lpt_x:6.1f}, whole chip {lpt_all:6.1f} | filled {filled:6.1f}")


if __name__ == "__main__":
    main()

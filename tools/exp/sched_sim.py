"""List-schedule simulation of k_vis work items from a recorded item
timeline (gpurun_out/item_times.npy, written by tools/exp/item_times.py).

Rows of the array are indexed by work item (the plan kernel's order); each
row holds start/end clocks (100 MHz), the item's info word (triangles,
slices) and the raster mid-point.  The simulation replays the measured
durations on `slots` concurrent workgroups (free slot -> next item, plus a
fixed dispatch gap) under several orders, to price a different item order
before building it:
  recorded   the plan's order (size classes, largest first)
  by_tris    triangles descending (finer classes)
  by_dur     measured duration descending (LPT bound)
Usage: python tools/exp/sched_sim.py [npy] [slots] [gap_us]"""
import heapq
import sys

import numpy as np


def simulate(durs, slots, gap):
    heap = [0.0] * slots
    end = 0.0
    for d in durs:
        t = heapq.heappop(heap)
        f = t + gap + d
        end = max(end, f)
        heapq.heappush(heap, f)
    return end


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/item_times.npy"
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    a = np.load(path)
    valid = a[:, 1] > a[:, 0]
    idx = np.nonzero(valid)[0]
    a = a[valid]
    dur = (a[:, 1].astype(np.int64) - a[:, 0].astype(np.int64)) / 100.0
    info = a[:, 2]
    ntri = (info & 0xFFFFFFFF).astype(np.int64)
    nsl = ((info >> 32) & 0xFFFF).astype(np.int64)
    span = (a[:, 1].max() - a[:, 0].min()) / 100.0
    print(f"items {len(a)} measured span {span:.1f} us, sum {dur.sum():.0f} us, "
          f"sum/slots {dur.sum() / slots:.1f} us, longest {dur.max():.1f} us")
    order = np.argsort(idx, kind="stable")
    key_tris = ntri + (nsl > 1) * 100000   # split slices first, as the plan does
    for name, o in (("recorded", order),
                    ("by_tris", np.argsort(-key_tris, kind="stable")),
                    ("by_dur", np.argsort(-dur, kind="stable"))):
        print(f"  {name:9s} slots {slots} gap {gap:.1f}: makespan {simulate(dur[o], slots, gap):.1f} us")


if __name__ == "__main__":
    main()

"""Debug (CPU): render_bwd group-slot occupancy from a hit dump (tools/dbg/hit_dump.py).

render_bwd runs one wave per tile as four 16-lane quadrant groups; a batch of B list entries takes
max_q(c_q) iterations, c_q = the batch's entries that contributed in quadrant q, so group-slots
past a quadrant's count idle.  Prints, for batch sizes B, the evaluated slots (4 x iterations),
the useful ones (sum c_q), the idle fraction, and the per-tile lower bound (each group walking its
whole tile list: max_q of the tile totals)."""
import sys

import numpy as np


def main(path):
    d = np.load(path)
    hit, ranges, work = d["hit"], d["ranges"], d["work"]
    bits = np.unpackbits(hit[:, None], axis=1, bitorder="little")[:, :4].astype(np.int64)  # (L, 4)
    cs = np.concatenate([np.zeros((1, 4), np.int64), np.cumsum(bits, 0)])
    useful = 0
    res = {}
    for B in (64, 96, 128, 192, 256):
        slots = 0
        for (a, _), w in zip(ranges, work):
            if w <= 0:
                continue
            starts = np.arange(0, w, B)
            ends = np.minimum(starts + B, w)
            cnt = cs[a + ends] - cs[a + starts]  # (batches, 4)
            slots += 4 * int(cnt.max(1).sum())
            if B == 64:
                useful += int(cnt.sum())
        res[B] = slots
    lb = 0
    for (a, _), w in zip(ranges, work):
        if w > 0:
            lb += 4 * int((cs[a + w] - cs[a]).max())
    print(f"useful group-slots {useful}")
    for B, s in res.items():
        print(f"B={B:4d}: slots {s}  idle {1 - useful / s:.3f}")
    print(f"per-tile bound: slots {lb}  idle {1 - useful / lb:.3f}")
    # launch tail: per-tile cost (iterations of the current B=64 scheme + a per-batch and per-tile
    # overhead, in iteration units), list-scheduled longest-first on S wave slots
    import heapq
    costs = []
    for (a, _), w in zip(ranges, work):
        if w <= 0:
            costs.append(2.0)
            continue
        starts = np.arange(0, w, 64)
        ends = np.minimum(starts + 64, w)
        cnt = cs[a + ends] - cs[a + starts]
        costs.append(float(cnt.max(1).sum()) + 4.0 * len(starts) + 8.0)
    costs = np.array(costs)
    print(f"tiles {len(costs)}  cost mean {costs.mean():.1f}  max {costs.max():.1f}  p99 {np.quantile(costs, .99):.1f}")
    for views in (1, 8):
        for S in (4096,):
            c = np.sort(np.tile(costs, views))[::-1]
            heap = [0.0] * S
            for x in c:
                t = heapq.heappop(heap)
                heapq.heappush(heap, t + x)
            ms = max(heap)
            print(f"views {views} slots {S}: makespan / ideal = {ms / (c.sum() / S):.3f} (max tile / ideal {c[0] / (c.sum() / S):.3f})")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hit_dump.npz")

"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite, the default output format):
per-family device time per step, GPU busy time (union of kernel intervals) and idle gaps over
the last STEPS steps of a bench run (one step = from one adam_kernel end to the next).

    python tools/trace_db.py gpurun_out/prof_X/run_results.db [--steps 20]
"""
import argparse
import collections
import sqlite3


def family(name: str) -> str:
    n = name.split("(")[0]
    for key, fam in (("conv3x3_pipe_kernel", "conv"), ("conv_first_fwd", "conv_first"),
                     ("wgrad_pipe", "wgrad"), ("wgrad_split", "wgrad"), ("wgrad_reduce", "wgrad_reduce"),
                     ("in_bwd_edge_kernelILi1", "edge_final"), ("in_bwd_edge_kernelILi2", "edge_first"),
                     ("in_bwd_edge_kernelILi3", "edge_first"),
                     ("in_bwd_kernel", "in_bwd_apply"), ("net_end", "net_end"), ("heads", "heads"),
                     ("adam", "adam"), ("pack", "pack"), ("loss", "loss")):
        if key in n:
            return fam
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="adam_kernel",
                    help="kernel that ends one iteration (c4 encoder-only batches: heads_fwd)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select d.start, d.end, s.kernel_name, d.stream_id, d.queue_id, s.arch_vgpr_count, "
                     "s.sgpr_count, s.private_segment_size from rocpd_kernel_dispatch d join "
                     "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    adam = [i for i, r in enumerate(rows) if a.marker in r[2]]
    i0, i1 = adam[-a.steps - 1], adam[-1]
    sel = rows[i0 + 1:i1 + 1]
    t0, t1 = rows[i0][1], rows[i1][1]
    wall = (t1 - t0) / a.steps / 1e6
    fam = collections.defaultdict(float)
    cnt = collections.Counter()
    for s, e, n, *_ in sel:
        fam[family(n)] += (e - s) / 1e6 / a.steps
        cnt[family(n)] += 1
    # busy = union of intervals
    busy, cur_s, cur_e = 0.0, None, None
    for s, e, *_ in sorted(sel):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"step wall {wall:.3f} ms   GPU busy (union) {busy / a.steps / 1e6:.3f} ms   "
          f"sum of kernel times {sum(fam.values()):.3f} ms")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {k:14s} {v:7.3f} ms/step  {cnt[k] // a.steps:4d} launches")
    big = collections.defaultdict(lambda: [0, 0.0, None])
    for s, e, n, _, _, vg, sg, ps in sel:
        d = big[n.split('(')[0]]
        d[0] += 1
        d[1] += (e - s) / 1e3
        d[2] = (vg, sg, ps)
    print("\nkernels (us per launch, launches/step, vgpr/sgpr/scratch):")
    for n, (k, us, res) in sorted(big.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {us / a.steps:8.1f} us/step {k // a.steps:3d}x {us / k:7.1f} us  {res}  {n[:110]}")


if __name__ == "__main__":
    main()

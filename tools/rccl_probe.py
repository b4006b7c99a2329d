"""RCCL all-reduce kernel resources on this GPU: a world-size-1 nccl group
all-reduces the step's two gradient buckets a few times; run under rocprofv3 --kernel-trace and
read the kernel's LDS / VGPR / SGPR / block size from the trace database.

    rocprofv3 --kernel-trace -d OUT -o run -- python3 tools/rccl_probe.py
    python3 tools/rccl_probe.py --db OUT/run_results.db
"""
import argparse
import os
import sqlite3


def report(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.kernel_name, max(d.group_segment_size), s.arch_vgpr_count, s.accum_vgpr_count, "
        "s.sgpr_count, s.private_segment_size, d.workgroup_size_x, d.grid_size_x, "
        "count(*), avg(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
        "on d.kernel_id = s.id group by s.kernel_name").fetchall()
    for n, lds, vg, ag, sg, ps, wg, gr, cnt, dur in rows:
        print(f"{n[:70]:70s} lds {lds:6d} B  vgpr {vg:3d} agpr {ag:3d} sgpr {sg:3d} scratch {ps:4d} "
              f"block {wg:4d} grid {gr:6d}  {cnt:3d}x {dur / 1e3:8.1f} us")


def run():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    buckets = [torch.ones(1_000_000, device=dev), torch.ones(850_000, device=dev)]   # ~7.4 MB
    for _ in range(10):
        for b in buckets:
            dist.all_reduce(b)
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("rccl probe done")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--db")
    a = ap.parse_args()
    report(a.db) if a.db else run()

"""Worker of tests/test_gpu_dist.py: one rank of a multi-GPU build whose collectives
run over torch.distributed/gloo on host copies (s3imph_host_comm), so several ranks
can share the one GPU of a test box.  The kernels, the routing, the segment layout and
the replicated tail are the production code; only the transport differs from RCCL."""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, world, port, shard, n_global, switch, result_q, mode="route"):
    try:
        for d in (os.path.join(ROOT, "s3-inv-db_amd"), os.path.join(ROOT, "oracle")):
            if d not in sys.path:
                sys.path.insert(0, d)
        os.environ["S3IMPH_DIST_SWITCH"] = str(switch)
        os.environ["S3IMPH_DIST_MODE"] = mode
        os.environ["S3IMPH_DIST_STRICT"] = "1"  # a bitmap build may not fall back to routing
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import s3imph
        dist.init_process_group("gloo", rank=rank, world_size=world)
        blob, offs, pos, key_base = shard
        n = len(offs) - 1
        ctx = s3imph.DistBuilder(0, None, rank, world, host_comm=True)
        cap = ctx.out_cap(n_global)
        pad = np.zeros(((len(blob) + 7) // 8) * 8 + 8, np.uint8)
        pad[:len(blob)] = blob
        d_blob = torch.from_numpy(pad).to("cuda:0")
        d_offs = torch.from_numpy(np.ascontiguousarray(offs, np.uint64).view(np.int64).copy()).to("cuda:0")
        d_pos = None
        if pos is not None:
            d_pos = torch.from_numpy(np.ascontiguousarray(pos, np.uint64).view(np.int64).copy()).to("cuda:0")
        d_fp = torch.zeros(max(cap, 1), dtype=torch.int64, device="cuda:0")
        d_po = torch.zeros(max(cap, 1), dtype=torch.int64, device="cuda:0")
        try:
            out_n, segs, info = ctx.build_shard(d_blob, d_offs, n, key_base, d_fp, d_po, cap, d_pos=d_pos)
        except s3imph.MPHFError as e:
            result_q.put((rank, "error", e.status, str(e)))
            dist.barrier()
            dist.destroy_process_group()
            return
        lf = d_fp[:out_n].cpu().numpy().view(np.uint64).copy()
        lp = d_po[:out_n].cpu().numpy().view(np.uint64).copy()
        result_q.put((rank, "ok", lf, lp, segs, ctx.mph_bin(), info))
        ctx.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - surfaced by the parent test
        result_q.put((rank, "exception", traceback.format_exc()))

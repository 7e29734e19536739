import os, sys, torch, torch.distributed as dist
import torch.multiprocessing as mp
def w(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29655")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    t = torch.full((8,), rank, dtype=torch.int32, device="cuda")
    s = torch.tensor([rank + 1], dtype=torch.int64, device="cuda")
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    gl = [torch.empty(8, dtype=torch.uint8, device="cuda") for _ in range(world)] if rank == 0 else None
    try:
        w_ = dist.gather(t.view(torch.uint8)[:8], gl, dst=0, async_op=True); w_.wait()
        print(rank, "gather ok", s.item(), [g.tolist()[:2] for g in gl] if gl else None, flush=True)
    except Exception as e:
        print(rank, "gather failed:", repr(e)[:300], flush=True)
    dist.barrier(); dist.destroy_process_group()
if __name__ == "__main__":
    mp.spawn(w, args=(2,), nprocs=2)

"""Round-6 probe: does RCCL run a world-2 group whose two ranks share the box's one GPU?  If it does, the extractor's
codes all-gather runs at world 2 on hardware (both ranks on cuda:0).  Launched by torch.distributed.run, 127.0.0.1."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
from audiotokenization_amd.extract import all_gather_codes  # noqa: E402

codes = (torch.arange(2 * 3 * 5, dtype=torch.int64).view(2, 3, 5) + 1000 * rank).to(torch.int16).cuda()
out = all_gather_codes(codes)
torch.cuda.synchronize()
ok = out.shape == (world, 2, 3, 5) and all(
    torch.equal(out[r].cpu(), (torch.arange(30).view(2, 3, 5) + 1000 * r).to(torch.int16)) for r in range(world))
print(f"rank {rank}: world {world} all_gather_codes over {dist.get_backend()} ok={ok}", flush=True)
dist.destroy_process_group()

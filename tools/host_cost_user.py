"""Host issue cost of the user-partitioned step (one-rank RCCL group, table sized as rank 0 of
WORLD ranks): host time of K step calls without synchronising vs the synchronised wall time.
Usage (GPU box): python tools/host_cost_user.py [WORLD]"""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

U, I, LAYERS, G, B, g = 138493, 27278, [128, 64, 32, 16], 64, 65536, 4
ew = int(sys.argv[1]) if len(sys.argv) > 1 else 8
torch.cuda.set_device(0)
sk = socket.socket()
sk.bind(("127.0.0.1", 0))
port = sk.getsockname()[1]
sk.close()
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
n_loc = (U + ew - 1) // ew
eng = NCFEngine(n_loc, I, LAYERS, G, max_batch=B)
eng.set_keras_weights(partition_keras_weights(initial_weights(U, I, LAYERS, G, seed=0), ew, 0))
dp = UserPartitionedDataParallel(eng)
gen = torch.Generator(device="cuda").manual_seed(1234)
pool = []
for _ in range(8):
    u = torch.randint(0, n_loc, (B // g,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(g)
    it = torch.randint(0, I, (B,), generator=gen, device="cuda", dtype=torch.int32)
    y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g)
    pool.append((u.contiguous(), it.contiguous(), y.contiguous()))


def step(i):
    u, it, y = pool[i % 8]
    nu, ni, _ = pool[(i + 1) % 8]
    dp.train_step(u, it, y, group=g, k=3, next_batch=(nu, ni))


for i in range(10):
    step(i)
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for i in range(K):
    step(10 + i)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host issue %.1f us/step, wall %.1f us/step" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
dist.destroy_process_group()

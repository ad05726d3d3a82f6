"""Experiment: host cost of the eager training step vs hipGraph replay (torch.cuda.graph),
config C or B, single table with deferred decay (or the dense sweep).  Checks that replay is
bitwise the eager step.  Usage (GPU box): python tools/exp_graph.py [lazy|dense] [C|B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT]

import torch  # noqa: E402

from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "lazy"
cfg = sys.argv[2] if len(sys.argv) > 2 else "C"
U, I, LAYERS, G, B, g = {"C": (138493, 27278, [128, 64, 32, 16], 64, 65536, 4),
                         "B": (6040, 3952, [64, 32, 16, 8], 8, 4095, 5)}[cfg]
print("config", cfg, mode, flush=True)
w0 = initial_weights(U, I, LAYERS, G, seed=0)


def make():
    e = NCFEngine(U, I, LAYERS, G, max_batch=B, lazy_adam=(mode == "lazy"))
    e.set_keras_weights(w0)
    return e


gen = torch.Generator(device="cuda").manual_seed(1234)
pool = []
for _ in range(8):
    u = torch.randint(0, U, (B // g,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(g)
    it = torch.randint(0, I, (B,), generator=gen, device="cuda", dtype=torch.int32)
    y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g)
    pool.append((u.contiguous(), it.contiguous(), y.contiguous()))
inv = 1.0 / B

a = make()
for i in range(10):
    a.train_step(*pool[i % 8], group=g, k=3, inv_batch=inv)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(50):
    a.train_step(*pool[i % 8], group=g, k=3, inv_batch=inv)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_eager = time.perf_counter() - t0
print("eager: host issue %.1f us/step, wall %.1f us/step" % (t_host / 50 * 1e6, t_eager / 50 * 1e6), flush=True)

# graphs: one per pool entry, captured on a side stream after a warmup there
b = make()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for i in range(3):
        b.train_step(*pool[i % 8], group=g, k=3, inv_batch=inv)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
graphs = []
for j in range(8):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        b.train_step(*pool[j], group=g, k=3, inv_batch=inv)
    graphs.append(gr)
torch.cuda.synchronize()
print("captured", flush=True)

# bitwise check: eager engine c vs graph replay on b, from identical states
c = make()
with torch.no_grad():
    for t_src, t_dst in ((b.emb, c.emb), (b.emb_m, c.emb_m), (b.emb_v, c.emb_v), (b.mlp, c.mlp),
                         (b.mlp_m, c.mlp_m), (b.mlp_v, c.mlp_v), (b.step, c.step), (b.stats, c.stats)):
        t_dst.copy_(t_src)
    if b.row_step is not None:
        c.row_step.copy_(b.row_step)
        c._dirty = True
for i in range(16):
    graphs[(3 + i) % 8].replay()
    c.train_step(*pool[(3 + i) % 8], group=g, k=3, inv_batch=inv)
b._dirty = True
b.flush()
c.flush()
torch.cuda.synchronize()
print("bitwise emb", torch.equal(b.emb, c.emb), "mlp", torch.equal(b.mlp, c.mlp), "m", torch.equal(b.emb_m, c.emb_m),
      flush=True)

torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(50):
    graphs[i % 8].replay()
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_graph = time.perf_counter() - t0
print("graph: host issue %.1f us/step, wall %.1f us/step" % (t_host / 50 * 1e6, t_graph / 50 * 1e6), flush=True)

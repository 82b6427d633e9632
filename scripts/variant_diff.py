"""Debug: print the records where a classify variant differs from production.

  python scripts/variant_diff.py <config> <variant> <frames>"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import pollnet_amd as pa
from pollnet_amd import tuning as tn
cfg, v, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
p = pa.rx.GenParams.for_config(cfg)
s = pa.gen_frames(p, n)
t = pa.gen_conn_table(p)
ctx = pa.RxContext(0)
ctx.set_conn_table(t)
fr = torch.from_numpy(s.reshape(-1)).cuda()
ref = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
res = torch.zeros_like(ref)
st = torch.cuda.current_stream()
ctx.classify(fr, 2048, 2, n, ref, st)
tn.classify_variant(ctx, fr, 2048, 2, n, res, st, v)
torch.cuda.synchronize()
a = ref.cpu().numpy().view(np.uint32).reshape(-1, 4)
b = res.cpu().numpy().view(np.uint32).reshape(-1, 4)
d = np.nonzero((a != b).any(1))[0]
print("differing", len(d), "of", n)
for i in d[:12]:
    print(i, [hex(x) for x in a[i]], [hex(x) for x in b[i]])

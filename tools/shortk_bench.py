import sys, math, torch
sys.path.insert(0, "/root/repo")
from simclr_amd.ops import _ext
from simclr_amd.ops.conv_hip import fwd_geom
ops = _ext.ops()
dev = torch.device("cuda", 0)
def timeit(fn, reps=20):
    fn(); s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); e.synchronize(); return s.elapsed_time(e) / reps * 1e3
for (N, H, C, Co) in [(1024, 8, 256, 1024), (1024, 8, 64, 1024), (1024, 4, 512, 2048), (1024, 8, 1024, 256)]:
    M = N * H * H
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, C, device=dev) / math.sqrt(C)).to(torch.bfloat16)
    y = torch.empty(N, H, H, Co, device=dev, dtype=torch.bfloat16)
    g = fwd_geom(N, H, H, C, H, H, 1, 1, 1, 0, Co)
    res = []
    for v in range(ops.igemm_nvariants()):
        if not ops.igemm_variant_ok(v, g, False, False): continue
        bm = ops.igemm_variant_bm(v)
        st = torch.empty((M // bm) * 2 * Co, device=dev)
        t0 = timeit(lambda: ops.igemm(x, w, y, None, None, g, None, None, 0, False, 0, None, None, v))
        t1 = timeit(lambda: ops.igemm(x, w, y, None, st, g, None, None, 0, False, 0, None, None, v))
        res.append((v, t0, t1))
    fl = 2.0 * M * Co * C
    by = 2.0 * (M * C + M * Co)
    best = min(res, key=lambda r: r[2])
    print(f"M={M} N={Co} K={C}: best v{best[0]} nostats {best[1]:.1f} stats {best[2]:.1f} us  ({fl/best[2]/1e6:.0f} TF, {by/best[2]/1e3:.0f} GB/s)  all: " + " ".join(f"v{v}:{a:.0f}/{b:.0f}" for v, a, b in res), flush=True)

"""Debug helper: 2 gloo ranks sharing cuda:0 vs 1 process — per-BN-layer batch mean / var
(recovered from the running statistics after one forward) and embeddings."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
N, W = 32, 2


def build(dev, fused):
    from simclr_amd.models.contrastive import ContrastiveModel
    from simclr_amd.parallel.flat import FlatParamStore
    torch.manual_seed(0)
    m = ContrastiveModel(base_cnn="resnet50", d=128, cifar_stem=True).to(dev)
    m.f.use_fused_stages = fused
    store = FlatParamStore(m, dev, shadow_dtype=torch.bfloat16)
    m.train()
    return m, store


def data():
    g = torch.Generator().manual_seed(11)
    return torch.rand(N * W, 8, 32, 32, generator=g), torch.rand(N * W, 8, 32, 32, generator=g)


def stats(m):
    out = {}
    for n, mod in m.named_modules():
        if hasattr(mod, "running_var"):
            out[n] = (mod.running_mean.float().cpu() / 0.1,
                      (mod.running_var.float().cpu() - 0.9) / 0.1)
    return out


def worker(rank, port, fused, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=W)
    from simclr_amd.parallel import state as pstate
    st = pstate.set_state(rank=rank, world_size=W, local_rank=0, group=dist.group.WORLD)
    st.device = dev
    pstate.make_stat_group(st)
    m, store = build(dev, fused)
    v0, v1 = data()
    sl = slice(rank * N, (rank + 1) * N)
    x = torch.cat([v0[sl], v1[sl]]).to(dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        z = m(x, segments=2)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"st": stats(m), "z": z.float().cpu()}, "/tmp/dbg_r0.pt")
    dist.barrier()
    dist.destroy_process_group()


def main():
    fused = len(sys.argv) > 1 and sys.argv[1] == "fused"
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, 29633, fused, None)) for r in range(W)]
    [p.start() for p in ps]
    [p.join() for p in ps]
    got = torch.load("/tmp/dbg_r0.pt", weights_only=True)
    from simclr_amd.parallel import state as pstate
    pstate.reset()
    dev = torch.device("cuda", 0)
    pstate.get().device = dev
    m, store = build(dev, fused)
    v0, v1 = data()
    x = torch.cat([v0, v1]).to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        z = m(x, segments=2)
    ref = stats(m)
    for k, (mu, var) in ref.items():
        gm, gv = got["st"][k]
        print(f"{k:40s} mean_err={float((gm - mu).norm() / (mu.norm() + 1e-9)):.4f} "
              f"var_err={float((gv - var).norm() / (var.norm() + 1e-9)):.4f}")
    zr = z.float().cpu()[:N]
    print("z rank0 view0 rows err", float((got["z"][:N] - zr).norm() / zr.norm()))


if __name__ == "__main__":
    main()

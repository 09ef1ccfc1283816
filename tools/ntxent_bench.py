"""NT-Xent kernel cost vs the number of columns (global negatives: W ranks x 1024 rows), one
GPU: normalise/transpose, forward (+finish/reduce) and both backward passes, R = 1024 local rows."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def timeit(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    R, D, n = 1024, 128, 512
    for W in (1, 2, 4, 8):
        C = W * R
        zall = torch.nn.functional.normalize(torch.randn(C, D, device=dev), dim=1)
        znT = torch.empty(D, C, device=dev)
        ops.nt_transpose(zall, znT)
        off = 0
        splits = ops.nt_fwd_splits(R, C)
        part = torch.empty(splits * R * 3, device=dev)
        lse = torch.empty(R, device=dev)
        rows = torch.empty(R, device=dev)
        out = torch.empty(1, device=dev)
        g = torch.ones(1, device=dev)

        def fwd():
            ops.nt_forward(znT, R, off, n, 2.0, part, splits, lse, rows)
            ops.nt_reduce_loss(rows, 1.0 / R, out)
        s_col, s_row = ops.nt_bwd_splits(C, R), ops.nt_bwd_splits(R, C)
        p2 = torch.empty(s_col * C * D, device=dev)
        dc = torch.empty(C, D, device=dev)
        p1 = torch.empty(s_row * R * D, device=dev)
        dr = torch.empty(R, D, device=dev)
        t_t = timeit(lambda: ops.nt_transpose(zall, znT))
        t_f = timeit(fwd)
        t_bc = timeit(lambda: ops.nt_backward_part(False, zall, znT, lse, R, off, n, 2.0, 1.0 / R,
                                                   g, p2, s_col, dc))
        t_br = timeit(lambda: ops.nt_backward_part(True, zall, znT, lse, R, off, n, 2.0, 1.0 / R,
                                                   g, p1, s_row, dr))
        fl = 2.0 * R * C * D
        print(f"W={W} cols={C}: transpose {t_t:.1f}  fwd {t_f:.1f}  bwd cols {t_bc:.1f}  "
              f"bwd rows {t_br:.1f} us  (fwd {fl / t_f / 1e6:.1f} TF/s, splits {splits}/{s_col}/{s_row})",
              flush=True)


if __name__ == "__main__":
    main()

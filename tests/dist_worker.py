"""One rank of the multi-process tests of jwave_amd.distributed (gloo on CPU, or
nccl on GPUs with --backend nccl).  Launched by tests/test_distributed.py as
separate processes; exits 0 when every case matches the single-process result.

On CPU the per-rank compute is the oracle (OracleBackend below — test
infrastructure); on GPU it is jwave_amd.distributed.HipBackend, and the
reference result is still the oracle on the full input.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
import jwave_amd as jw  # noqa: E402
from jwave_amd import distributed as D  # noqa: E402


class OracleBackend:
    """Per-rank compute on the CPU oracle (tests only)."""

    def rows(self, x, w, level, forward, kind="fwt"):
        return torch.from_numpy(oracle.batch(kind, forward, w, x.numpy(), level))

    def cols(self, x, w, level, forward, kind="fwt"):
        y = oracle.batch(kind, forward, w, np.ascontiguousarray(x.numpy().T), level)
        return torch.from_numpy(np.ascontiguousarray(y.T))

    def modwt_fwd(self, x, w, J):
        return torch.from_numpy(oracle.modwt_forward(w, x.numpy(), J))

    def modwt_inv(self, c, w):
        return torch.from_numpy(oracle.modwt_inverse(w, c.numpy()))

    def modwt_fwd_ld(self, x, c, n, J, w):
        c[:, :n] = torch.from_numpy(oracle.modwt_forward(w, x[:n].numpy(), J))

    def modwt_inv_ld(self, c, col0, n, x, w):
        x[:n] = torch.from_numpy(oracle.modwt_inverse(w, np.ascontiguousarray(
            c[:, col0:col0 + n].numpy())))


class ChunkedOracleBackend(OracleBackend):
    """OracleBackend plus the chunked row passes HipBackend has (the oracle's
    rows, laid out as jwv_fwt_rows_seg_* lay them out: [cols/seg][rows][seg]),
    so the gloo runs exercise the exchange without pack / unpack copies."""

    @staticmethod
    def _check_seg(seg):
        # the native entries' rule (capi.cpp check_seg)
        if seg < 2 or seg & (seg - 1):
            raise ValueError("seg must be a power of two >= 2 dividing cols")

    def rows_to_chunks(self, x, w, level, seg):
        self._check_seg(seg)
        y = oracle.batch("fwt", True, w, x.numpy(), level)
        rows, cols = y.shape
        return torch.from_numpy(np.ascontiguousarray(
            y.reshape(rows, cols // seg, seg).transpose(1, 0, 2)))

    def chunks_to_rows(self, y, w, level):
        nch, rows, seg = y.shape
        self._check_seg(seg)
        plain = np.ascontiguousarray(y.numpy().transpose(1, 0, 2).reshape(rows, nch * seg))
        return torch.from_numpy(oracle.batch("fwt", False, w, plain, level))


def same(a, b, what):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    if a.shape != b.shape or not np.array_equal(a, b):
        d = np.abs(a - b).max() if a.shape == b.shape else "shape %s vs %s" % (a.shape, b.shape)
        raise AssertionError("%s: mismatch (%s)" % (what, d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--backend", default="gloo")
    a = ap.parse_args()
    if a.backend == "nccl":
        torch.cuda.set_device(a.rank)
        dev = torch.device("cuda", a.rank)
        be = D.HipBackend(jw.Context(a.rank))
    else:
        dev = torch.device("cpu")
        be = OracleBackend()
    dist.init_process_group(a.backend, init_method="tcp://127.0.0.1:%d" % a.port,
                            rank=a.rank, world_size=a.world)
    W, r = a.world, a.rank

    def put(arr):
        return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)

    # ---- batches (config 4 shape, small): contiguous row blocks, no collective
    for kind, wname, total, n, lev in (("wpt", "Symlet8", 7, 256, 3), ("fwt", "Daubechies4", 5, 64, 6)):
        w = jw.by_class(wname)
        full = oracle.java_random_doubles(42, total * n).reshape(total, n)
        s, c = D.shard_range(total, W, r)
        y = D.batch_forward(put(full[s:s + c]), w, lev, be, kind)
        yg = D.gather_rows(y.cpu() if a.backend == "gloo" else y, total)
        same(yg, oracle.batch(kind, True, w, full, lev), "%s batch fwd" % kind)
        xr = D.batch_reverse(y, w, lev, be, kind)
        same(D.gather_rows(xr, total), oracle.batch(kind, False, w,
                                                    oracle.batch(kind, True, w, full, lev), lev),
             "%s batch rev" % kind)

    # ---- 2-D: row pass, all-to-all transpose, column pass (FWT: chunked row
    # passes and, on gloo, also the packing fallback; WPT: the fallback)
    bes2 = [be] if a.backend == "nccl" else [ChunkedOracleBackend(), be]
    for kind, wname, rows, cols, lm, ln in (
            ("fwt", "Daubechies8", 64, 128, 6, 7), ("fwt", "Haar1", 32, 16, 2, 3),
            ("fwt", "Daubechies4", 128, 64, 5, 0), ("fwt", "Daubechies4", 8, 4096, 3, 12),
            ("wpt", "Symlet8", 64, 64, 4, 5),
            # cols == W: one-column chunks take the plain pass + packing copy
            ("fwt", "Haar1", 4, 2, 2, 1)):
        if rows % W or cols % W:
            continue
        w = jw.by_class(wname)
        full = oracle.java_random_doubles(123456789, rows * cols).reshape(rows, cols)
        rw = rows // W
        ref = oracle.transform_2d(kind, True, w, full, lm, ln)
        for b2 in bes2:
            tag = "%s %s %dx%d %s" % (kind, wname, rows, cols, type(b2).__name__)
            yc = D.forward_2d(put(full[r * rw:(r + 1) * rw]), rows, cols, w, lm, ln, b2, kind=kind)
            same(D.gather_cols(yc), ref, "2d fwd " + tag)
            xr = D.reverse_2d(yc, rows, cols, w, lm, ln, b2, kind=kind)
            same(D.gather_rows(xr, rows), oracle.transform_2d(kind, False, w, ref, lm, ln),
                 "2d rev " + tag)

    # ---- MODWT of one long signal: ring halo exchange
    for wname, n, J in (("Daubechies4", 1000, 5), ("Haar1", 1001, 3), ("Daubechies8", 4096, 4)):
        w = jw.by_class(wname)
        full = oracle.java_random_doubles(42, n)
        s, c = D.shard_range(n, W, r)
        cf = D.modwt_forward(put(full[s:s + c]), n, w, J, be)
        ref = oracle.modwt_forward(w, full, J)
        got = D.gather_rows(cf.t().contiguous(), n).t()
        same(got, ref, "modwt fwd %s n=%d" % (wname, n))
        xr = D.modwt_inverse(cf, n, w, be)
        same(D.gather_rows(xr, n), oracle.modwt_inverse(w, ref), "modwt inv %s n=%d" % (wname, n))
        # the same through the persistent strided buffers (no slice copies)
        sh = D.ModwtShard(n, w, J, dev)
        assert (sh.start, sh.n) == (s, c)
        sh.x.copy_(put(full[s:s + c]))
        for rep in range(2):  # reused buffers: the second call must not see the first's halos
            cs = sh.forward(be)
            same(D.gather_rows(cs.t().contiguous(), n).t(), ref, "shard fwd %s #%d" % (wname, rep))
            same(D.gather_rows(sh.inverse(be).contiguous(), n), oracle.modwt_inverse(w, ref),
                 "shard inv %s #%d" % (wname, rep))

    dist.barrier()
    dist.destroy_process_group()
    print("rank %d OK" % r, flush=True)


if __name__ == "__main__":
    main()

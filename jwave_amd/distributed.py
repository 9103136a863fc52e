"""Multi-GPU sharding of the hot path: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).

What shards, and how:

* Batches of signals (FWT/WPT batch, config 4): contiguous row blocks per rank,
  no data-path collective (`shard_range`, `batch_forward/reverse`).
* 2-D FWT (config 3, BasicTransform.java:361-474): row block per rank -> row
  pass -> all-to-all transpose of [R/W x C/W] blocks -> column pass on the
  [R][C/W] slab.  The row kernels write (forward) / read (reverse) the
  all-to-all chunk layout directly (jwv_fwt_rows_seg_*), so no pack / unpack
  pass touches HBM around the exchange.  The forward result stays in that column-slab layout, which
  is exactly what the sharded reverse consumes; `gather_cols` assembles it.
* MODWT of one long signal (config 5, MODWTTransform.java:256-375): contiguous
  slices; forward receives a left halo of H = (L-1)(2^J - 1) samples from its
  ring predecessor, inverse a right halo of H columns of all J+1 rows from its
  successor (one send/recv pair per direction).  Each rank then runs the
  ordinary single-GPU transform on its extended slice as a periodic signal of
  length n_local + H; the wrap only reaches the H outputs that are dropped, and
  every kept output is summed from the same values in the same order, so the
  sharded result is bit-identical to the single-GPU one.
* One long 1-D FWT (config 2) does not shard: replicas only.

Per-rank compute goes through a backend object; `HipBackend` (the only one in
the package) calls the C ABI on the rank's GPU.  Tests substitute the CPU
oracle to exercise the exchange logic with gloo on CPU.
"""
import torch
import torch.distributed as dist

from . import transforms as T


def shard_range(total, world, rank):
    """Contiguous block split: (start, count) of rank `rank`; the first
    total % world ranks get one extra item."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


class HipBackend:
    """Per-rank compute on this rank's GPU through libjwave_hip.so."""

    def __init__(self, ctx=None):
        self.ctx = ctx

    def rows(self, x, w, level, forward, kind="fwt"):
        f = T.fwt_forward if forward else T.fwt_reverse
        return f(x, w, level, self.ctx, kind=kind)

    def cols(self, x, w, level, forward, kind="fwt"):
        # [R][cw] slab: transform along dim 0 (outer = 1, inner = cw)
        return T.transform_axis(x, w, level, 0, forward, self.ctx, kind=kind)

    def rows_to_chunks(self, x, w, level, seg):
        """FWT row pass writing the all-to-all send layout [C/seg][rw][seg]."""
        return T.fwt_rows_to_chunks(x, w, level, seg, self.ctx)

    def chunks_to_rows(self, y, w, level):
        """FWT reverse row pass reading the all-to-all receive layout."""
        return T.fwt_chunks_to_rows(y, w, level, self.ctx)

    def modwt_fwd(self, x, w, J):
        return T.modwt_forward(x, w, J, self.ctx)

    def modwt_inv(self, c, w):
        return T.modwt_inverse(c, w, self.ctx)

    def modwt_fwd_ld(self, x, c, n, J, w):
        """forwardMODWT of x[:n] into the rows of c (row stride c.stride(0)),
        columns [0, n); jwv_modwt_fwd_ld_f64_dev."""
        T.modwt_forward_ld(x, c, n, J, w, self.ctx)

    def modwt_inv_ld(self, c, col0, n, x, w):
        """inverseMODWT of the columns [col0, col0 + n) of the rows of c into
        x[:n]; jwv_modwt_inv_ld_f64_dev."""
        T.modwt_inverse_ld(c, col0, n, x, w, self.ctx)


def _world(group):
    return dist.get_world_size(group), dist.get_rank(group)


# --------------------------------------------------------------- batches
def batch_forward(x_local, w, level, backend, kind="fwt"):
    """This rank's block of a sharded batch ([b_local][n]); no collective."""
    return backend.rows(x_local, w, level, True, kind)


def batch_reverse(y_local, w, level, backend, kind="fwt"):
    return backend.rows(y_local, w, level, False, kind)


def gather_rows(local, total, group=None):
    """All-gather of contiguous row blocks (uneven blocks padded) -> [total][...]."""
    W, _ = _world(group)
    counts = [shard_range(total, W, r)[1] for r in range(W)]
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], 0)


# --------------------------------------------------------------- 2-D FWT
def _check_2d(rows, cols, W):
    if rows % W or cols % W:
        raise ValueError("sharded 2-D transform needs rows and cols divisible by the world size "
                         "(%d x %d over %d ranks)" % (rows, cols, W))


def _segmentable(cw):
    """The segmented row passes (jwv_fwt_rows_seg_*) take chunks of a power of
    two >= 2 columns (capi.cpp check_seg); one-column chunks (cols == W) take
    the plain pass and one packing copy."""
    return cw >= 2 and (cw & (cw - 1)) == 0


def _rows_to_send(x_rows, w, level, W, backend, kind):
    """Row pass whose result is the all-to-all send buffer [W][rw][cw] (chunk
    j -> rank j).  A backend with rows_to_chunks (HipBackend, FWT) writes
    that layout from the row kernels; otherwise the plain rows are packed
    with one copy."""
    rw, C = x_rows.shape
    cw = C // W
    if kind == "fwt" and _segmentable(cw) and hasattr(backend, "rows_to_chunks"):
        return backend.rows_to_chunks(x_rows, w, level, cw)
    a = backend.rows(x_rows, w, level, True, kind)
    return a.reshape(rw, W, cw).permute(1, 0, 2).contiguous()


def _recv_to_rows(recv, w, level, backend, kind):
    """Reverse row pass reading the all-to-all receive buffer [W][rw][cw]
    (chunk j = my rows of rank j's columns) in place where the backend can."""
    W, rw, cw = recv.shape
    if kind == "fwt" and _segmentable(cw) and hasattr(backend, "chunks_to_rows"):
        return backend.chunks_to_rows(recv, w, level)
    return backend.rows(recv.permute(1, 0, 2).reshape(rw, W * cw), w, level, False, kind)


def _exchange(send, group):
    """all-to-all of the [W][rw][cw] chunks: chunk j -> rank j, chunk i <- rank i."""
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv


def forward_2d(x_rows, rows, cols, w, lvl_m, lvl_n, backend, group=None, kind="fwt"):
    """BasicTransform.forward(double[][], lvlM, lvlN) (BasicTransform.java:361-399)
    sharded: x_rows = this rank's [rows/W][cols] block; returns this rank's
    [rows][cols/W] column slab of the result.  HBM passes per rank besides the
    two transforms: none -- the row pass writes the send chunks, the column
    pass reads the receive buffer as the [rows][cols/W] slab it is."""
    W, _ = _world(group)
    _check_2d(rows, cols, W)
    recv = _exchange(_rows_to_send(x_rows, w, lvl_n, W, backend, kind), group)
    return backend.cols(recv.reshape(rows, cols // W), w, lvl_m, True, kind)


def reverse_2d(y_cols, rows, cols, w, lvl_m, lvl_n, backend, group=None, kind="fwt"):
    """BasicTransform.reverse(double[][], lvlM, lvlN) (BasicTransform.java:436-474)
    sharded: y_cols = this rank's [rows][cols/W] slab; returns its
    [rows/W][cols] row block of the reconstruction.  The column pass's output
    is the send buffer as is; the row pass reads the receive chunks."""
    W, _ = _world(group)
    _check_2d(rows, cols, W)
    b = backend.cols(y_cols, w, lvl_m, False, kind)
    recv = _exchange(b.reshape(W, rows // W, cols // W), group)
    return _recv_to_rows(recv, w, lvl_n, backend, kind)


def gather_cols(slab, group=None):
    """[R][cw] column slabs of all ranks -> the full [R][C] matrix."""
    W, _ = _world(group)
    parts = [torch.empty_like(slab) for _ in range(W)]
    dist.all_gather(parts, slab.contiguous(), group=group)
    return torch.cat(parts, 1)


# --------------------------------------------------------------- MODWT
def modwt_halo(L, J):
    """Samples of context a level-J MODWT output needs on one side:
    sum_j (L-1) 2^(j-1) (MODWTTransform.java:618-630 upsampled filter spans)."""
    return (L - 1) * ((1 << J) - 1)


def _ring_exchange(send, recv, to, frm, group):
    reqs = [dist.isend(send.contiguous(), to, group=group),
            dist.irecv(recv, frm, group=group)]
    for r in reqs:
        r.wait()


def _check_modwt(n_global, J, counts, H):
    # the reference's own checks (MODWTTransform.java:257-282) on the global N
    T._check_modwt_levels(n_global, J)
    if min(counts) < H:
        raise ValueError("sharded MODWT needs every slice >= the halo (%d < %d)"
                         % (min(counts), H))


class ModwtShard:
    """One rank's buffers of a sharded MODWT of one long signal
    (MODWTTransform.java:256-375), laid out so that neither direction copies
    a slice: H = modwt_halo(L, J).

    * xe = [left halo (H) | x_local (n)]: the forward's extended periodic
      signal; the ring exchange receives the halo straight into xe[:H].
    * c: J+1 rows at stride ld = H + n + H.  The forward writes columns
      [0, H + n); the kept coefficients are columns [H, H + n) (c_local);
      the inverse's right halo -- the successor's first H kept columns --
      lands in columns [H + n, 2H + n), and the inverse reads [H, 2H + n).
    * xr: the inverse's n + H outputs; the first n are this rank's slice.
    The wrap of each extended periodic transform reaches only the H outputs
    that are dropped, and every kept output sums the same values in the same
    order as the unsharded transform, so kept results are bit-identical."""

    def __init__(self, n_global, w, J, device, group=None):
        dtype = torch.float64  # the C-ABI _ld entries address these as doubles
        W, rank = _world(group)
        counts = [shard_range(n_global, W, r)[1] for r in range(W)]
        self.H = H = modwt_halo(w.mother_wavelength, J)
        _check_modwt(n_global, J, counts, H)
        self.W, self.rank, self.group = W, rank, group
        self.n, self.J, self.w = counts[rank], J, w
        self.start = shard_range(n_global, W, rank)[0]
        n = self.n
        self.ld = ld = H + n + H
        self.xe = torch.empty(H + n, dtype=dtype, device=device)
        self.x = self.xe[H:]
        self.c = torch.empty((J + 1, ld), dtype=dtype, device=device)
        self.xr = torch.empty(n + H, dtype=dtype, device=device)
        self._send = torch.empty((J + 1, H), dtype=dtype, device=device)
        self._recv = torch.empty((J + 1, H), dtype=dtype, device=device)

    @property
    def coeffs(self):
        """This rank's [J+1][n] block of [W_1 .. W_J, V_J] (a strided view)."""
        return self.c[:, self.H:self.H + self.n]

    def exchange_forward(self):
        """Left halo: my last H samples -> successor, predecessor's -> xe[:H]."""
        if self.W > 1:
            _ring_exchange(self.xe[self.n:self.n + self.H], self.xe[:self.H],
                           (self.rank + 1) % self.W, (self.rank - 1) % self.W, self.group)
        else:  # one rank: the periodic wrap of the whole signal
            self.xe[:self.H].copy_(self.x[self.n - self.H:])

    def exchange_inverse(self):
        """Right halo: my first H kept columns -> predecessor, successor's ->
        columns [H + n, 2H + n) (via a (J+1) x H staging pair)."""
        H, n = self.H, self.n
        self._send.copy_(self.c[:, H:2 * H])
        if self.W > 1:
            _ring_exchange(self._send, self._recv, (self.rank - 1) % self.W,
                           (self.rank + 1) % self.W, self.group)
            self.c[:, H + n:2 * H + n].copy_(self._recv)
        else:
            self.c[:, H + n:2 * H + n].copy_(self._send)

    def forward(self, backend):
        self.exchange_forward()
        backend.modwt_fwd_ld(self.xe, self.c, self.H + self.n, self.J, self.w)
        return self.coeffs

    def inverse(self, backend):
        self.exchange_inverse()
        backend.modwt_inv_ld(self.c, self.H, self.n + self.H, self.xr, self.w)
        return self.xr[:self.n]


def modwt_forward(x_local, n_global, w, J, backend, group=None):
    """forwardMODWT of one signal sharded in contiguous slices
    (shard_range(n_global, W, rank)): returns this rank's [J+1][n_local] block
    of [W_1 .. W_J, V_J]."""
    W, rank = _world(group)
    counts = [shard_range(n_global, W, r)[1] for r in range(W)]
    H = modwt_halo(w.mother_wavelength, J)
    _check_modwt(n_global, J, counts, H)
    if W == 1:
        return backend.modwt_fwd(x_local, w, J)
    halo = torch.empty(H, dtype=x_local.dtype, device=x_local.device)
    # my last H samples -> successor's left halo; predecessor's last H -> mine
    _ring_exchange(x_local[-H:], halo, (rank + 1) % W, (rank - 1) % W, group)
    ext = torch.cat([halo, x_local])
    c = backend.modwt_fwd(ext, w, J)
    return c[:, H:].contiguous()


def modwt_inverse(c_local, n_global, w, backend, group=None):
    """inverseMODWT of a sharded coefficient block [J+1][n_local]: returns this
    rank's slice of the reconstruction."""
    W, rank = _world(group)
    J = c_local.shape[0] - 1
    counts = [shard_range(n_global, W, r)[1] for r in range(W)]
    H = modwt_halo(w.mother_wavelength, J)
    _check_modwt(n_global, J, counts, H)
    if W == 1:
        return backend.modwt_inv(c_local, w)
    halo = torch.empty((J + 1, H), dtype=c_local.dtype, device=c_local.device)
    # my first H columns -> predecessor's right halo; successor's -> mine
    _ring_exchange(c_local[:, :H], halo, (rank - 1) % W, (rank + 1) % W, group)
    ext = torch.cat([c_local, halo], 1).contiguous()
    x = backend.modwt_inv(ext, w)
    return x[:c_local.shape[1]].contiguous()

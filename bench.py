#!/usr/bin/env python3
"""Benchmark of the JWave hot path on MI355X (BASELINE.json metric).

Default workload (config 2, the metric's configuration): 1-D FWT, Daubechies4,
N = 2^24 fp64, full depth (24 levels).  One step = forward + reverse of one
signal resident in HBM.  With N GPUs every rank transforms its own signal: the
single-signal FWT does not shard ("replicas", weak scaling).
Other workloads (--workload):
  fwt2d : config 3, Daubechies8 8192x8192, 13x13 levels (rows+columns), fwd+rev
  wpt   : config 4, Symlet8 6 levels, 4096 x 65536 signals sharded over ranks
          (strong scaling), fwd+rev
  modwt : config 5, Daubechies4 J=8, N = 10^7, forwardMODWT + inverseMODWT

The default run also measures config 4 as a secondary object
("batched_wpt_strong"): the 4096 signals split over the ranks, data-resident
per-rank compute between barriers, and, separately, the time to
gather every rank's coefficients to rank 0 over RCCL.

Launch: `python bench.py --gpus N` starts its N ranks itself (a
torch.distributed.run child; this parent process never touches the GPU), or
runs as one rank of an external torch.distributed.run.

Prints ONE JSON line (rank 0).  value = samples transformed per second over
all ranks (forward and reverse each count N samples); hbm_gbps = algorithmic
bytes / time.  "roofline" is for the dominant kernel, timed with hipEvents
recorded around its launches on its own stream during a second timed region.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec, an FMA counts 2 flops
WORKLOADS = ["fwt1d", "fwt2d", "wpt", "modwt"]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--warmup-seconds", type=float, default=0.25,
                   help="minimum wall time of the warmup steps (after the first W)")
    p.add_argument("--workload", default="fwt1d", choices=WORKLOADS)
    p.add_argument("--math", default="exact", choices=["exact", "fma"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--config-cpu-seconds", type=float, default=3.0,
                   help="CPU-leg budget of each config object in the default line")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the config-4 strong-scaling object of the default run")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher/timing plumbing only: gloo on CPU, a placeholder host step, "
                        "no transform (tests)")
    return p.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` outside torch.distributed.run: start N ranks as ONE child
    torch.distributed.run (one process per GPU) and return its exit code.
    This process imports nothing that initialises the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


class Dist:
    def __init__(self, gpus, dry):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = dry
        if self.world != gpus:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (run `python bench.py --gpus %d` "
                             "alone, or as one rank of torch.distributed.run --nproc-per-node %d)"
                             % (gpus, self.world, gpus, gpus))
        self.pg = None
        self.dev = None
        if not dry:
            import torch
            torch.cuda.set_device(self.local)
            self.dev = torch.device("cuda", self.local)
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if dry:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=self.dev)
            self.pg = dist

    def sync(self):
        if not self.dry:
            import torch
            torch.cuda.synchronize()

    def barrier(self):
        if self.pg:
            if self.dry:
                self.pg.barrier()
            else:
                self.pg.barrier(device_ids=[self.local])

    def _reduce(self, v, op):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev if not self.dry else "cpu")
        self.pg.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v):
        return self._reduce(v, self.pg.ReduceOp.MAX if self.pg else None)

    def sum(self, v):
        return self._reduce(v, self.pg.ReduceOp.SUM if self.pg else None)

    def broadcast_taps(self, cls):
        """Rank 0 owns the filter bank; every rank receives it over RCCL
        (the taps/config broadcast of SURVEY §8e)."""
        import torch
        import jwave_amd as jw
        w = jw.by_class(cls)
        if not self.pg:
            return w
        L = w.mother_wavelength
        buf = torch.zeros(4 * L + 3, dtype=torch.float64, device=self.dev)
        if self.rank == 0:
            buf[:] = torch.tensor(w.lo + w.hi + w.lo_r + w.hi_r +
                                  [w.reverse_scale, L, w.transform_wavelength], dtype=torch.float64)
        self.pg.broadcast(buf, src=0)
        v = buf.cpu().tolist()
        w.lo, w.hi, w.lo_r, w.hi_r = v[:L], v[L:2 * L], v[2 * L:3 * L], v[3 * L:4 * L]
        w.reverse_scale = v[4 * L]
        return w

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


# ------------------------------------------------------------------ workloads
class PlaceholderBackend:
    """--dry-run per-rank "compute" on CPU tensors: copies of the right shapes,
    so the sharded workloads' exchanges (jwave_amd.distributed: all-to-all
    transposes, MODWT ring halos) run for real over gloo without a GPU."""

    def rows(self, x, w, level, forward, kind="fwt"):
        return x.clone()

    def cols(self, x, w, level, forward, kind="fwt"):
        return x.clone()

    def modwt_fwd_ld(self, x, c, n, J, w):
        c[:, :n] = x[:n]

    def modwt_inv_ld(self, c, col0, n, x, w):
        x[:n] = c[0, col0:col0 + n]


# Algorithmic FP64 flops per sample per direction of each workload (a mul and
# an add counted apart, as EXACT mode issues them):
#   fwt1d  Daubechies4, L = 8, full depth: 2L per level-input sample, the
#          levels' inputs sum to ~2N -> 4L;
#   fwt2d  Daubechies8, L = 16: the same for the row pass and the column pass;
#   wpt    Symlet8, L = 16, 6 levels over the whole row each: 6 x 2L;
#   modwt  Daubechies4, L = 8, J = 8: per level and output L taps on each of
#          two inputs (forward: V and W outputs; inverse: V and W inputs) -> 4L.
FLOPS_PER_SAMPLE = {"fwt1d": 4 * 8, "fwt2d": 2 * 4 * 16, "wpt": 6 * 2 * 16, "modwt": 8 * 4 * 8}


def step_bounds(workload, math, bytes_per_step, samples_per_step, ms_per_step):
    """Both floors of one step at one GPU: the algorithmic HBM bytes at the HBM
    peak and the algorithmic FP64 flops at the FP64 issue ceiling (EXACT: mul
    and add are separate instructions, so half the FMA-counted peak).  'frac'
    is the larger floor over the measured step; 'frac_of_sum' the two floors
    added (a step whose memory and FP64 phases do not overlap at all sits at
    1.0 of it).  samples_per_step counts both directions, like the line's
    value."""
    fps = FLOPS_PER_SAMPLE.get(workload)
    if fps is None or not ms_per_step:
        return None
    flops = fps * samples_per_step
    ceil = FP64_PEAK_TFLOPS / 2 if math == "exact" else FP64_PEAK_TFLOPS
    hbm_ms = bytes_per_step / (HBM_PEAK_GBPS * 1e9) * 1e3
    fp_ms = flops / (ceil * 1e12) * 1e3
    return {"hbm_floor_ms": round(hbm_ms, 4), "fp64_floor_ms": round(fp_ms, 4),
            "flops_per_step": flops, "fp64_ceiling_tflops": ceil,
            "bound": "hbm" if hbm_ms >= fp_ms else "fp64",
            "frac": round(max(hbm_ms, fp_ms) / ms_per_step, 4),
            "frac_of_sum": round((hbm_ms + fp_ms) / ms_per_step, 4)}


def setup_dry(args, d):
    """--dry-run: a placeholder host step (no transform, no GPU) so the
    launcher, barriers and max-over-ranks timing can be tested on CPU; the
    sharded workloads (fwt2d, modwt at world > 1) run their real exchanges
    around placeholder compute."""
    import numpy as np
    if d.world > 1 and args.workload in ("fwt2d", "modwt"):
        return setup_sharded(args, d, None, PlaceholderBackend(), "cpu", small=True)
    a = np.random.default_rng(d.rank).random(1 << 16)
    b = np.empty_like(a)

    def step():
        np.copyto(b, a)

    return dict(ctx=None, step=step, check=lambda: 0.0, samples=2 * a.size, bytes=32.0 * a.size,
                metric="dry-run (launcher test, no transform)",
                config={"workload": "dry-run", "parallelism": "ranks x%d" % d.world},
                scaling="weak", cpu=None)


def setup_sharded(args, d, ctx, backend, device, small=False):
    """Configs 3 and 5 split over the ranks as SURVEY 8(e) / DESIGN 7 shard
    them (strong scaling: one problem, fixed total size):
      fwt2d: row block per rank -> row pass -> all-to-all transpose -> column
             pass on the [R][C/W] slab; the reverse mirrors it
             (ParallelTransform.java:70-126's row/column structure);
      modwt: contiguous slices of the 10^7-sample signal, one ring halo
             exchange per direction (MODWTTransform.java:256-375).
    'exchange' times the data-path collectives alone on the same buffers."""
    import numpy as np
    import torch
    from jwave_amd import distributed as D
    import jwave_amd as jw
    W, rank = d.world, d.rank
    if args.workload == "fwt2d":
        r = c = 256 if small else 8192
        lev = r.bit_length() - 1
        w = jw.by_class("Daubechies8") if small else d.broadcast_taps("Daubechies8")
        rw = r // W
        full = np.random.default_rng(42).random((r, c))
        x = torch.from_numpy(np.ascontiguousarray(full[rank * rw:(rank + 1) * rw])).to(device)
        del full
        st = {}

        def step():
            slab = D.forward_2d(x, r, c, w, lev, lev, backend)
            st["xr"] = D.reverse_2d(slab, r, c, w, lev, lev, backend)

        a = torch.empty((W, rw, c // W), dtype=torch.float64, device=device)
        b = torch.empty((W, rw, c // W), dtype=torch.float64, device=device)

        def exchange():  # the two all-to-alls alone (send buffers written in place)
            D._exchange(a, None)
            D._exchange(b, None)

        return dict(ctx=ctx, step=step, exchange=exchange,
                    check=lambda: float((st["xr"] - x).abs().max().item()),
                    samples=2 * rw * c, bytes=2 * 32.0 * rw * c,
                    metric="samples/s, 2D FWT Daubechies8 8192x8192 fp64",
                    config={"workload": "fwt2d: 2D FWT Daubechies8 %dx%d, %dx%d levels, "
                                        "forward+reverse per step, row blocks -> all-to-all -> "
                                        "column slabs" % (r, c, lev, lev), "math": args.math,
                            "parallelism": "sharded x%d (strong)" % W},
                    scaling="strong", cpu=None if small else ("fwt2d", w))
    n, J = (20_000 if small else 10_000_000), 8
    w = jw.by_class("Daubechies4") if small else d.broadcast_taps("Daubechies4")
    sh = D.ModwtShard(n, w, J, device)
    xs = np.random.default_rng(42).random(n)[sh.start:sh.start + sh.n]
    sh.x.copy_(torch.from_numpy(xs).to(device))

    def step():
        sh.forward(backend)
        sh.inverse(backend)

    def exchange():
        sh.exchange_forward()
        sh.exchange_inverse()

    return dict(ctx=ctx, step=step, exchange=exchange,
                check=lambda: float((sh.xr[:sh.n] - sh.x).abs().max().item()),
                samples=2 * sh.n, bytes=2 * 80.0 * sh.n,
                metric="samples/s, MODWT Daubechies4 J=8 N=1e7 fp64",
                config={"workload": "modwt: Daubechies4, J=8, N=%d, forwardMODWT+inverseMODWT "
                                    "per step, contiguous slices + ring halo (%d samples)"
                                    % (n, sh.H), "math": args.math,
                        "parallelism": "sharded x%d (strong)" % W},
                scaling="strong", cpu=None if small else ("modwt", w))


def setup(args, d, workload=None):
    """-> dict(step=callable, samples, bytes per step, metric, config, cpu spec)."""
    import numpy as np
    import torch
    import jwave_amd as jw
    from jwave_amd import _lib as L
    from jwave_amd.transforms import _TapsHolder

    workload = workload or args.workload
    ctx = jw.Context(d.local, args.math)
    ctx.set_stream(torch.cuda.current_stream(d.dev).cuda_stream)
    lib = L.lib()
    h = ctx.handle
    rng = np.random.default_rng(42 + d.rank)

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(d.dev)

    def p(t):
        return ctypes.c_void_p(t.data_ptr())

    def chk(rc):
        if rc:
            raise RuntimeError(lib.jwv_last_error(h).decode())

    if workload == "fwt1d":
        n = 1 << 24
        w = d.broadcast_taps("Daubechies4")
        t = _TapsHolder.of(w)
        x = dev(rng.random(n))
        y = torch.empty_like(x)
        xr = torch.empty_like(x)

        def step():
            chk(lib.jwv_fwt_fwd_f64_dev(p(x), p(y), n, 24, t, h))
            chk(lib.jwv_fwt_rev_f64_dev(p(y), p(xr), n, 24, t, h))

        def check():
            return float((xr - x).abs().max().item())

        return dict(ctx=ctx, step=step, check=check, samples=2 * n, bytes=2 * 16.0 * n,
                    metric="samples/s + achieved HBM GB/s, 1D FWT Daubechies4 N=2^24 fp64",
                    config={"workload": "fwt1d: 1D FWT Daubechies4, N=2^24, full depth "
                                        "(24 levels), forward+reverse per step",
                            "wavelet": "Daubechies4", "n": n, "levels": 24, "batch_per_gpu": 1,
                            "directions_per_step": 2, "math": args.math,
                            "parallelism": "replicas x%d (one signal per GPU)" % d.world},
                    scaling="weak", cpu=("fwt1d", w))
    if workload in ("fwt2d", "modwt") and d.world > 1:
        from jwave_amd import distributed as D
        args.workload = workload
        return setup_sharded(args, d, ctx, D.HipBackend(ctx), d.dev)
    if workload == "fwt2d":
        r = c = 8192
        w = d.broadcast_taps("Daubechies8")
        t = _TapsHolder.of(w)
        x = dev(rng.random(r * c))
        y = torch.empty_like(x)
        xr = torch.empty_like(x)

        def step():
            chk(lib.jwv_fwt2d_fwd_f64_dev(p(x), p(y), r, c, 13, 13, t, h))
            chk(lib.jwv_fwt2d_rev_f64_dev(p(y), p(xr), r, c, 13, 13, t, h))

        def check():
            return float((xr - x).abs().max().item())

        return dict(ctx=ctx, step=step, check=check, samples=2 * r * c, bytes=2 * 32.0 * r * c,
                    metric="samples/s, 2D FWT Daubechies8 8192x8192 fp64",
                    config={"workload": "fwt2d: 2D FWT Daubechies8 8192x8192, 13x13 levels, "
                                        "forward+reverse per step", "math": args.math,
                            "parallelism": "replicas x%d" % d.world},
                    scaling="weak", cpu=("fwt2d", w))
    if workload == "wpt":
        total, n = 4096, 1 << 16
        b = total // d.world
        w = d.broadcast_taps("Symlet8")
        t = _TapsHolder.of(w)
        x = torch.rand(b, n, dtype=torch.float64, device=d.dev,
                       generator=torch.Generator(device=d.dev).manual_seed(42 + d.rank))
        y = torch.empty_like(x)
        xr = torch.empty_like(x)

        def step():
            chk(lib.jwv_wpt_fwd_batch_f64_dev(p(x), p(y), b, n, n, 6, t, h))
            chk(lib.jwv_wpt_rev_batch_f64_dev(p(y), p(xr), b, n, n, 6, t, h))

        def check():
            return float((xr - x).abs().max().item())

        return dict(ctx=ctx, step=step, check=check, samples=2 * b * n, bytes=2 * 16.0 * b * n,
                    metric="samples/s, batched WPT Symlet8 6 levels 4096x65536 fp64",
                    config={"workload": "wpt: Symlet8, 6 levels, %d signals x 65536 "
                                        "(%d per GPU), forward+reverse per step" % (total, b),
                            "math": args.math, "parallelism": "batch shards x%d" % d.world},
                    scaling="strong", cpu=("wpt", w), coef=y, signals=b, n=n,
                    # 6 levels x (L = 16 taps x 2 filters) MACs per pair = 2 x 16 x 2
                    # flops per sample per level: FP64-bound too
                    flops_per_sample=6 * 2 * 16 * 2 / 2)
    # modwt
    n, J = 10_000_000, 8
    w = d.broadcast_taps("Daubechies4")
    t = _TapsHolder.of(w)
    x = dev(rng.random(n))
    cf = torch.empty((J + 1) * n, dtype=torch.float64, device=d.dev)
    xr = torch.empty_like(x)

    def step():
        chk(lib.jwv_modwt_fwd_f64_dev(p(x), p(cf), n, J, t, h))
        chk(lib.jwv_modwt_inv_f64_dev(p(cf), p(xr), n, J, t, h))

    def check():
        return float((xr - x).abs().max().item())

    return dict(ctx=ctx, step=step, check=check, samples=2 * n, bytes=2 * 80.0 * n,
                metric="samples/s, MODWT Daubechies4 J=8 N=1e7 fp64",
                config={"workload": "modwt: Daubechies4, J=8, N=10^7, forwardMODWT+"
                                    "inverseMODWT per step", "math": args.math,
                        "parallelism": "replicas x%d" % d.world},
                scaling="weak", cpu=("modwt", w))


# ------------------------------------------------------------- CPU baseline
def _host():
    """(threads we may use, nproc, CPU model).  On the GPU box the process's
    CPU share is 16 threads (os.cpu_count() shows the whole machine)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return max(1, min(16, avail)), os.cpu_count() or 1, model


def cpu_baseline(spec, seconds):
    """The reference's CPU path, restated by the oracle (C, -O2
    -ffp-contract=off), timed on this host on a bounded sample of the same
    workload:
      fwt1d: single thread (JWave has no parallel 1-D FWT, FastWaveletTransform.java:90-97);
      fwt2d: ParallelTransform's rows -> join -> columns split over all host
             threads (ParallelTransform.java:70-126), the full 8192x8192 matrix;
      wpt:   signal-level parallel batch over all host threads
             (ParallelizationOpportunityTest.java:80-98) on a sample of the signals;
      modwt: single-thread DIRECT including the zero taps of the upsampled
             filters (MODWTTransform.java:677-716) on a non-power-of-2 prefix
             (DIRECT work per sample does not depend on N)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    kind, w = spec
    threads, nproc, model = _host()
    rng = np.random.default_rng(42)
    reps, t0 = 0, time.perf_counter()
    if kind == "fwt1d":
        n, used = 1 << 24, 1
        x = rng.random(n)
        while True:
            y = oracle.fwt_forward(w, x, 24)
            oracle.fwt_reverse(w, y, 24)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 50:
                break
        samples = 2.0 * n * reps
        what = ("%d x (forward+reverse) of one Daubechies4 N=2^24 full-depth signal, single "
                "thread" % reps)
    elif kind == "fwt2d":
        r = c = 8192
        used = threads
        x = rng.random((r, c))
        while True:
            y = oracle.transform_2d_par("fwt", True, w, x, 13, 13, used)
            oracle.transform_2d_par("fwt", False, w, y, 13, 13, used)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 5:
                break
        samples = 2.0 * r * c * reps
        what = ("%d x (forward+reverse) of Daubechies8 8192x8192 13x13, ParallelTransform "
                "rows/join/columns on %d threads" % (reps, used))
    elif kind == "wpt":
        nsig, n = 64, 1 << 16
        used = threads
        x = rng.random((nsig, n))
        while True:
            y = oracle.batch_par("wpt", True, w, x, 6, used)
            oracle.batch_par("wpt", False, w, y, 6, used)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 50:
                break
        samples = 2.0 * nsig * n * reps
        what = ("%d x (forward+reverse) of %d Symlet8 L6 signals x 65536 (sample of the 4096), "
                "signal-level parallel on %d threads" % (reps, nsig, used))
    else:  # modwt
        n, J, used = 131071, 8, 1
        x = rng.random(n)
        while True:
            cf = oracle.modwt_forward(w, x, J, sparse=False)
            oracle.modwt_inverse(w, cf, sparse=False)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 50:
                break
        samples = 2.0 * n * reps
        what = ("%d x (forwardMODWT+inverseMODWT) Daubechies4 J=8 DIRECT (zero taps included) "
                "on N=131071 (prefix sample; per-sample work as at N=10^7), single thread" % reps)
    return {"value": samples / el, "unit": "samples/s", "cores": used, "kind": "port",
            "sample": "%s, oracle/jwave_oracle*.c (-O2 -ffp-contract=off), %.1f s" % (what, el),
            "host": {"nproc": nproc, "cpu_model": model, "threads_allowed": threads}}


# --------------------------------------------------------------- roofline
def load_traffic(workload, kernel, math, lib_sha=None):
    """HBM bytes per launch of `kernel` in `workload` from the committed
    rocprofv3 PMC summaries (profiles/pmc_*.json, key "workload:kernel/math"),
    preferring a summary taken with the library being measured (its
    build.lib_sha256, recorded by tools/pmc_traffic.py); (None, None, None)
    when no summary covers that workload's kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    found = []
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        ent = d.get("kernels", {}).get("%s:%s/%s" % (workload, kernel, math))
        if ent and ent.get("hbm_bytes_per_launch"):
            found.append((float(ent["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT),
                          (d.get("build") or {}).get("lib_sha256")))
    for t in found:
        if lib_sha and t[2] == lib_sha:
            return t
    return found[0] if found else (None, None, None)


def timed(d, step, steps, issue=None):
    """Seconds for `steps` steps between barrier + device syncs; `issue`
    (a list) receives the host time spent enqueueing them (when it is close
    to the total, the host, not the GPU, sets the pace)."""
    d.barrier()
    d.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t1 = time.perf_counter()
    d.sync()
    d.barrier()
    if issue is not None:
        issue.append(t1 - t0)
    return time.perf_counter() - t0


def secondary_wpt(args, d):
    """Config 4 (Symlet8 L6, 4096 x 65536) split over the ranks: data-resident
    per-rank compute between barriers (max over ranks), then the gather of
    every rank's coefficients to rank 0 over RCCL, timed separately."""
    import torch
    W = setup(args, d, "wpt")
    # the same warmup floor as the timed configs (--warmup-seconds): the
    # round-5 driver line timed 4 steps after 2 and read 4.48 ms/step against
    # 4.245 in configs.config4_wpt
    for _ in range(2):
        W["step"]()
    d.sync()
    t0 = time.perf_counter()
    while d.max(time.perf_counter() - t0) < args.warmup_seconds:
        for _ in range(4):
            W["step"]()
        d.sync()
    steps = max(5, min(10, args.steps // 2))
    el = d.max(timed(d, W["step"], steps))
    total = W["samples"] * steps * d.world
    out = {"workload": W["config"]["workload"], "scaling": "strong", "n_gpus": d.world,
           "value": round(total / el, 1), "unit": "samples/s",
           "ms_per_step": round(el / steps * 1e3, 4), "steps": steps,
           "hbm_gbps": round(W["bytes"] * steps * d.world / el / 1e9, 1),
           "roundtrip_max_abs_err": d.max(W["check"]())}
    y = W["coef"]
    nbytes = y.numel() * 8
    if d.pg:
        import torch.distributed as dist
        bufs = [torch.empty_like(y) for _ in range(d.world - 1)] if d.rank == 0 else None

        def gather():
            if d.rank == 0:
                ops = [dist.P2POp(dist.irecv, bufs[r - 1], r) for r in range(1, d.world)]
            else:
                ops = [dist.P2POp(dist.isend, y, 0)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()

        gather()  # warm the P2P channels
        g = d.max(timed(d, gather, 1))
        out["gather_to_rank0_ms"] = round(g * 1e3, 3)
        out["gather_bytes"] = nbytes * (d.world - 1)
        out["gather_GBps_into_rank0"] = round(nbytes * (d.world - 1) / g / 1e9, 1)
    else:
        out["gather_to_rank0_ms"] = 0.0
    del W
    return out


def _affinity():
    """CPUs this process may run on (the box's share, not its nproc)."""
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def host_entry(args, d, reps=5):
    """SURVEY 8(d) secondary reporting: the drop-in host path end to end
    (Transform.forward(double[]) -> FastWaveletTransform, Transform.java:81-90):
    jwv_fwt_fwd_f64 + jwv_fwt_rev_f64 on host arrays of config 2, pageable
    (what a JNI caller without staging hands over) and page-locked
    (jwv_host_alloc: what the JNI shim copies Java arrays into), next to the
    bare PCIe time of the same bytes (pinned H2D + D2H of the 128 MiB array,
    per direction)."""
    import numpy as np
    import torch
    import jwave_amd as jw
    from jwave_amd import _lib as L
    from jwave_amd.transforms import _TapsHolder
    lib = L.lib()
    n = 1 << 24
    w = jw.by_class("Daubechies4")
    t = _TapsHolder.of(w)
    ctx = jw.Context(d.local, args.math)
    h = ctx.handle
    dp = ctypes.POINTER(ctypes.c_double)
    x = np.random.default_rng(7).random(n)
    y = np.empty(n)
    xr = np.empty(n)

    def step(a, b, c):
        for fn, src, dst in ((lib.jwv_fwt_fwd_f64, a, b), (lib.jwv_fwt_rev_f64, b, c)):
            if fn(src.ctypes.data_as(dp), dst.ctypes.data_as(dp), n, 24, t, h):
                raise RuntimeError(lib.jwv_last_error(h).decode())

    def per_step(f):
        f()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        return (time.perf_counter() - t0) / reps * 1e3

    out = {"workload": "config 2 (D4, N=2^24, full depth) through the host-pointer entries, "
                       "forward + reverse per step", "steps": reps}
    st = (ctypes.c_double * 6)()
    step(x, y, xr)  # first touch of the outputs, ring allocation
    lib.jwv_ctx_stage_stats(h, st, 1)
    out["pageable_ms_per_step"] = round(per_step(lambda: step(x, y, xr)), 3)
    lib.jwv_ctx_stage_stats(h, st, 1)
    nst = reps + 1  # per_step runs one untimed call first
    # the pinned ring (capi.cpp PinRing): host copy threads, their time and
    # the time they waited for the DMA engine, per step; overlap = the share
    # of the host copies that ran while a DMA was in flight
    cp = (st[0] + st[3]) / nst * 1e3
    wt = (st[1] + st[2]) / nst * 1e3
    nbytes = (st[4] + st[5]) / nst
    out["ring"] = {"copy_threads": lib.jwv_host_copy_threads(),
                   "host_copy_ms_per_step": round(cp, 3),
                   "host_copy_GBps": round(nbytes / (cp * 1e-3) / 1e9, 1) if cp > 0 else None,
                   "dma_wait_ms_per_step": round(wt, 3), "bytes_per_step": nbytes,
                   "cpu_affinity": _affinity()}
    err = float(np.abs(xr - x).max())
    bufs = [ctypes.c_void_p() for _ in range(3)]
    try:
        for b in bufs:
            if lib.jwv_host_alloc(h, n * 8, ctypes.byref(b)):
                raise RuntimeError(lib.jwv_last_error(h).decode())
        px, py, pr = [np.ctypeslib.as_array((ctypes.c_double * n).from_address(b.value))
                      for b in bufs]
        px[:] = x
        out["pinned_ms_per_step"] = round(per_step(lambda: step(px, py, pr)), 3)
        err = max(err, float(np.abs(pr - x).max()))
        # the bare link: the same bytes H2D then D2H, pinned, per direction
        dev = torch.empty(n, dtype=torch.float64, device=d.dev)
        tx = torch.from_numpy(px)
        ty = torch.from_numpy(py)

        def link():
            dev.copy_(tx, non_blocking=True)
            ty.copy_(dev, non_blocking=True)
            torch.cuda.synchronize(d.dev)

        pcie = per_step(link)
    finally:
        for b in bufs:
            if b.value:
                lib.jwv_host_free(h, b)
    ctx.close()
    out["pcie_h2d_plus_d2h_ms_per_direction"] = round(pcie, 3)
    out["pinned_over_pcie"] = round(out["pinned_ms_per_step"] / (2 * pcie), 3)
    out["pageable_over_pcie"] = round(out["pageable_ms_per_step"] / (2 * pcie), 3)
    out["pinned_GBps"] = round(2 * 16.0 * n / (out["pinned_ms_per_step"] * 1e-3) / 1e9, 1)
    out["roundtrip_max_abs_err"] = err
    return out


def measure(args, d, W, workload, steps, warmup, math):
    """Warmup (W steps, then at least --warmup-seconds), timed region A
    (the metric, no events), timed region B (every launch evented in its own
    dispatch packet) -> the dominant kind's roofline."""
    step, ctx = W["step"], W["ctx"]
    # W warmup steps, and at least --warmup-seconds of them: MI355X needs
    # ~10 ms of sustained work before its step time settles (config 2, one
    # box: 110-123 us/step over the first 60 steps, 106 us after), so a short
    # W would time the ramp, not the kernels.  The line reports both counts.
    for _ in range(warmup):
        step()
    wsteps = warmup
    d.sync()
    t0 = time.perf_counter()
    # chunks of 16 steps; every rank takes the same decision (the sharded
    # steps hold collectives)
    while d.max(time.perf_counter() - t0) < args.warmup_seconds and wsteps < 100000:
        for _ in range(16):
            step()
        wsteps += 16
        d.sync()
    # nothing between the warmup and region A: an idle gap (the round-trip
    # check's first torch kernels load their code objects, ~0.15 s) lets the
    # clocks drop, and region A then times the ramp back (config 3, r04q
    # trace: 1.26 ms steady steps, 1.52 / 1.44 / ... after the gap).  The
    # check runs after the timed regions, on the same step's outputs.
    # timed region A: the metric (no events)
    issue = []
    el = d.max(timed(d, step, steps, issue))
    r = {"el": el, "issue": issue[0], "wsteps": wsteps, "prof": {}, "tb": None, "roof": None,
         "fp64": None}
    if ctx is not None:
        # timed region B: same steps, every launch carrying start/stop events
        # in its own dispatch packet (hipExtLaunchKernelGGL: the kernel's
        # execution alone, as rocprofv3 times it) -> roofline.achieved of the
        # dominant kind.  Eventing only that kind's launches timed them 7-8%
        # longer than rocprofv3 (config 2 / 5, r04m).
        ctx.profile_select(None)
        ctx.profile(True)
        r["tb"] = d.max(timed(d, step, steps))
        ctx.profile(False)
        prof = r["prof"] = ctx.profile_read()
        kname = max(prof.items(), key=lambda kv: kv[1]["total_ms"])[0]
        ks = prof[kname]
        avg_ms = ks["total_ms"] / ks["launches"]
        bytes_per_launch = ks["bytes"] / ks["launches"]
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        from jwave_amd import _lib as _L
        lib_sha = _L.provenance().get("lib_sha256")
        traffic, tsrc, tsha = load_traffic(workload, kname, math, lib_sha)
        r["roof"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "kernel": kname, "avg_launch_us": round(avg_ms * 1e3, 2),
                     "algorithmic_bytes_per_launch": bytes_per_launch, "launches": ks["launches"]}
        if tsrc:
            r["roof"]["traffic_source"] = tsrc
            r["roof"]["traffic_lib_sha256"] = tsha
            r["roof"]["traffic_same_lib"] = bool(lib_sha) and tsha == lib_sha
        if W.get("flops_per_sample"):
            # second bound: algorithmic FP64 flops of the
            # dominant launch over its time; EXACT mode issues mul and add
            # separately, so its ceiling is half the FMA-counted peak
            fl = W["flops_per_sample"] * bytes_per_launch / 16.0
            tf = fl / (avg_ms * 1e-3) / 1e12
            r["fp64"] = {"bound": "fp64", "achieved": round(tf, 2), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tf / FP64_PEAK_TFLOPS, 4),
                         "flops_per_launch": fl,
                         "exact_mode_ceiling": FP64_PEAK_TFLOPS / 2 if math == "exact" else None}
    return r


def kernels_of(prof):
    """Per-kind averages of region B (every launch evented in its packet)."""
    return {k: {"launches": v["launches"], "avg_us": round(v["total_ms"] * 1e3 / v["launches"], 2),
                "GBps": round(v["bytes"] / (v["total_ms"] * 1e-3) / 1e9, 1)}
            for k, v in prof.items()}


def secondary_configs(args, d):
    """BASELINE configs 3, 4 (EXACT and FMA) and 5 at one GPU, each timed as
    its own --workload run would time it (same warmup, regions A and B), in
    compact form.  One object per config, {"error": ...} if one fails.
    Returns (objects, CPU-baseline specs): main() times the CPU legs after
    every GPU leg."""
    import copy
    out, specs = {}, {}
    for key, wl, math in (("config3_fwt2d", "fwt2d", "exact"), ("config4_wpt", "wpt", "exact"),
                          ("config4_wpt_fma", "wpt", "fma"), ("config5_modwt", "modwt", "exact")):
        a = copy.copy(args)
        a.math = math
        try:
            W = setup(a, d, wl)
            r = measure(a, d, W, wl, args.steps, args.warmup, math)
            el = r["el"]
            o = {"workload": W["config"]["workload"], "math": math,
                 "ms_per_step": round(el / args.steps * 1e3, 4),
                 "value": round(W["samples"] * args.steps * d.world / el, 1), "unit": "samples/s",
                 "hbm_gbps": round(W["bytes"] * args.steps * d.world / el / 1e9, 1),
                 "steps": args.steps, "warmup_steps_run": r["wsteps"],
                 "roofline": r["roof"], "kernels_profiled_pass": kernels_of(r["prof"]),
                 "roundtrip_max_abs_err": W["check"]()}
            if r["fp64"]:
                o["roofline_fp64"] = r["fp64"]
            o["step_bounds"] = step_bounds(wl, math, W["bytes"], W["samples"],
                                           el / args.steps * 1e3)
            specs[key] = W["cpu"]
            W["ctx"].close()
            del W
        except Exception as e:  # one config's failure must not void the metric line
            o = {"workload": wl, "math": math, "error": "%s: %s" % (type(e).__name__, e)}
        out[key] = o
    return out, specs


def config_cpu_baselines(configs, specs, seconds):
    """Bounded CPU legs of the driver-timed config objects (rank 0, after every
    GPU leg): the same restated reference paths as cpu_baseline() -- config 3
    on the full matrix over the host threads, config 4 on a 64-signal sample,
    config 5 on the 131071-sample DIRECT prefix.  The FMA object shares config
    4's leg: the reference has one CPU path for both."""
    done = {}
    for key, o in configs.items():
        spec = specs.get(key)
        if spec is None or "error" in o:
            continue
        wl = spec[0]
        if wl in done:
            o["cpu_baseline"] = dict(done[wl][1], same_as=done[wl][0])
            continue
        try:
            o["cpu_baseline"] = cpu_baseline(spec, seconds)
            done[wl] = (key, o["cpu_baseline"])
        except Exception as e:
            o["cpu_baseline"] = {"error": "%s: %s" % (type(e).__name__, e)}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    d = Dist(args.gpus, args.dry_run)
    W = setup_dry(args, d) if args.dry_run else setup(args, d)
    ctx = W["ctx"]
    r = measure(args, d, W, args.workload, args.steps, args.warmup, args.math)
    el, wsteps, prof, tb = r["el"], r["wsteps"], r["prof"], r["tb"]
    out_roof, out_fp64, issue = r["roof"], r["fp64"], [r["issue"]]

    exch = None
    if W.get("exchange"):
        # the data-path collectives of the sharded step alone, same buffers
        W["exchange"]()
        exch = d.max(timed(d, W["exchange"], args.steps)) / args.steps * 1e3
    world = d.world
    value = W["samples"] * args.steps * world / el
    gbps = W["bytes"] * args.steps * world / el / 1e9
    err = W["check"]()
    kernels = kernels_of(prof if ctx is not None else {})
    out = {"metric": W["metric"], "value": round(value, 1), "unit": "samples/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "warmup_steps_run": wsteps, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
           "host_issue_ms_per_step": round(issue[0] / args.steps * 1e3, 4),
           "scaling": W["scaling"], "vs_baseline": None,
           "dtype": "f64", "data": "synthetic (uniform [0,1) doubles, seed 42+rank)",
           "config": W["config"], "hbm_gbps": round(gbps, 1), "roofline": out_roof,
           "kernels_profiled_pass": kernels, "roundtrip_max_abs_err": err}
    if not args.dry_run:
        from jwave_amd import _lib
        out["build"] = _lib.provenance()  # the library measured: its sources and digest
    if tb is not None:
        out["ms_per_step_with_events"] = round(tb / args.steps * 1e3, 4)
    if exch is not None:
        out["exchange_ms_per_step"] = round(exch, 4)
    if out_fp64:
        out["roofline_fp64"] = out_fp64
    if not args.dry_run:
        out["step_bounds"] = step_bounds(args.workload, args.math, W["bytes"], W["samples"],
                                         el / args.steps * 1e3)
    if (not args.dry_run and args.workload == "fwt1d" and not args.no_secondary):
        out["batched_wpt_strong"] = secondary_wpt(args, d)
        if d.rank == 0:
            out["host_entry"] = host_entry(args, d)
        # configs 3-5 at one GPU in the driver-timed line (their sharded
        # multi-GPU forms are --workload runs)
        if d.world == 1:
            out["configs"], cfg_specs = secondary_configs(args, d)
    # the reference's CPU path on this node's host cores, in the same run, at
    # every world size (rank 0, after every GPU leg)
    if d.rank == 0 and W["cpu"] and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(W["cpu"], args.cpu_seconds)
        if "configs" in out:
            config_cpu_baselines(out["configs"], cfg_specs, args.config_cpu_seconds)
    else:
        out["cpu_baseline"] = None
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()

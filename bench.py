#!/usr/bin/env python3
"""Benchmark of the JWave hot path on MI355X (BASELINE.json metric).

Default workload (config 2, the metric's configuration): 1-D FWT, Daubechies4,
N = 2^24 fp64, full depth (24 levels).  One step = forward + reverse of one
signal resident in HBM.  With N GPUs (torch.distributed.run, one rank per GPU,
RCCL) every rank transforms its own signal: the single-signal FWT does not
shard ("replicas", weak scaling).  Other workloads (--workload):
  fwt2d : config 3, Daubechies8 8192x8192, 13x13 levels (rows+columns), fwd+rev
  wpt   : config 4, Symlet8 6 levels, 4096 x 65536 signals sharded over ranks
          (strong scaling), fwd+rev
  modwt : config 5, Daubechies4 J=8, N = 10^7, forwardMODWT + inverseMODWT

Prints ONE JSON line (rank 0).  value = samples transformed per second over
all ranks (forward and reverse each count N samples); hbm_gbps = algorithmic
bytes / time.  "roofline" is for the dominant kernel, timed with hipEvents
recorded around its launches on its own stream during the timed region.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec (an FMA counts 2 flops)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (spec), SURVEY §8d


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="fwt1d", choices=["fwt1d", "fwt2d", "wpt", "modwt"])
    p.add_argument("--math", default="exact", choices=["exact", "fma"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


class Dist:
    def __init__(self, gpus):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != gpus and gpus != 1:
            raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (gpus, self.world))
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl", device_id=self.dev)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier(device_ids=[self.local])

    def max(self, v):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

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
def setup(args, d):
    """-> dict(step=callable, samples_per_step, bytes_per_step, desc...)."""
    import numpy as np
    import torch
    import jwave_amd as jw
    from jwave_amd import _lib as L
    from jwave_amd.transforms import _TapsHolder

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

    if args.workload == "fwt1d":
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
                    scaling="weak", cpu=("fwt", w, n, 24))
    if args.workload == "fwt2d":
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
                    scaling="weak", cpu=None)
    if args.workload == "wpt":
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
                    scaling="strong", cpu=None,
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
                scaling="weak", cpu=None)


def cpu_baseline(spec, seconds):
    """The oracle's restatement of the reference CPU path, single thread, on a
    bounded sample of the same workload (JWave has no parallel 1-D FWT:
    FastWaveletTransform.java:90-97)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    kind, w, n, lev = spec
    x = np.random.default_rng(42).random(n)
    reps, t0 = 0, time.perf_counter()
    while True:
        y = oracle.fwt_forward(w, x, lev)
        oracle.fwt_reverse(w, y, lev)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 50:
            break
    return {"value": 2.0 * n * reps / el, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": "%d x (forward+reverse) of the same Daubechies4 N=2^24 full-depth signal, "
                      "single thread, oracle/jwave_oracle.c (-O2 -ffp-contract=off), %.1f s"
                      % (reps, el)}


def load_traffic(kernel, math):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        ent = d.get("kernels", {}).get("%s/%s" % (kernel, math))
        if ent and ent.get("hbm_bytes_per_launch"):
            return float(ent["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


def main():
    args = parse()
    import torch
    d = Dist(args.gpus)
    W = setup(args, d)
    step, ctx = W["step"], W["ctx"]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    err = W["check"]()

    # which kernel kind dominates: one short profiled pass (not timed)
    ctx.profile_select(None)
    ctx.profile(True)
    for _ in range(3):
        step()
    ctx.profile(False)
    pre = ctx.profile_read()
    kname = max(pre.items(), key=lambda kv: kv[1]["total_ms"])[0]

    # timed region A: the metric (no events)
    d.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    d.barrier()
    t1 = time.perf_counter()

    # timed region B: same steps, hipEvents around the dominant kernel's
    # launches only (on its stream) -> roofline.achieved
    ctx.profile_select(kname)
    ctx.profile(True)
    d.barrier()
    torch.cuda.synchronize()
    tb0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    d.barrier()
    tb1 = time.perf_counter()
    ctx.profile(False)
    prof = ctx.profile_read()
    ctx.profile_select(None)

    el = d.max(t1 - t0)
    world = d.world
    samples = W["samples"] * args.steps * world
    value = samples / el
    gbps = W["bytes"] * args.steps * world / el / 1e9

    ks = prof[kname]
    avg_ms = ks["total_ms"] / ks["launches"]
    bytes_per_launch = ks["bytes"] / ks["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic, tsrc = load_traffic(kname, args.math)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": kname,
            "avg_launch_us": round(avg_ms * 1e3, 2), "algorithmic_bytes_per_launch": bytes_per_launch,
            "launches": ks["launches"]}
    if tsrc:
        roof["traffic_source"] = tsrc
    if W.get("flops_per_sample"):
        # second bound: algorithmic FP64 flops of the
        # dominant launch over its time; EXACT mode issues mul and add
        # separately, so its ceiling is half the FMA-counted peak
        fl = W["flops_per_sample"] * bytes_per_launch / 16.0
        tf = fl / (avg_ms * 1e-3) / 1e12
        out_fp64 = {"bound": "fp64", "achieved": round(tf, 2), "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tf / FP64_PEAK_TFLOPS, 4),
                    "flops_per_launch": fl,
                    "exact_mode_ceiling": FP64_PEAK_TFLOPS / 2 if args.math == "exact" else None}
    else:
        out_fp64 = None
    kernels = {k: {"launches": v["launches"], "avg_us": round(v["total_ms"] * 1e3 / v["launches"], 2),
                   "GBps": round(v["bytes"] / (v["total_ms"] * 1e-3) / 1e9, 1)}
               for k, v in pre.items()}

    out = {"metric": W["metric"], "value": round(value, 1), "unit": "samples/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": W["scaling"], "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (uniform [0,1) doubles, seed 42+rank)",
           "config": W["config"], "hbm_gbps": round(gbps, 1), "roofline": roof,
           "kernels_profiled_pass": kernels, "roundtrip_max_abs_err": err,
           "ms_per_step_with_events": round(d.max(tb1 - tb0) / args.steps * 1e3, 4)}
    if out_fp64:
        out["roofline_fp64"] = out_fp64
    if d.rank == 0 and world == 1 and W["cpu"] and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(W["cpu"], args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()

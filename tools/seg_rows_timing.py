"""Per-rank cost of the sharded 2-D transform's row passes around the
all-to-all (jwave_amd/distributed.py), round 5 vs round 4, on one GPU:

  r04: plain row pass + pack   (reshape/permute/contiguous)  /  unpack + plain reverse
  r05: chunked row pass         (jwv_fwt_rows_seg_fwd)        /  jwv_fwt_rows_seg_rev

for the row block one rank of an 8192 x 8192 Daubechies8 problem holds at
W = 2, 4, 8 (rows = 8192 / W, seg = 8192 / W), full level.  Prints one line
per (W, direction) with the median ms of each form and checks both forms give
identical values.  Usage: python tools/seg_rows_timing.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import jwave_amd as jw  # noqa: E402
from jwave_amd import transforms as T  # noqa: E402


def med_ms(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ctx = jw.Context(0, "exact")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    w = jw.by_class("Daubechies8")
    C = 8192
    lev = 13
    g = torch.Generator(device="cuda").manual_seed(1)
    for W in (2, 4, 8):
        rw, cw = C // W, C // W
        x = torch.rand((rw, C), dtype=torch.float64, device="cuda", generator=g)

        def r04_fwd():
            a = T.fwt_forward(x, w, lev, ctx)
            return a.reshape(rw, W, cw).permute(1, 0, 2).contiguous()

        def r05_fwd():
            return T.fwt_rows_to_chunks(x, w, lev, cw, ctx)

        s4, s5 = r04_fwd(), r05_fwd()
        assert torch.equal(s4, s5), "forward forms differ"
        t4, t5 = med_ms(r04_fwd, reps), med_ms(r05_fwd, reps)
        gb = 16.0 * rw * C / 1e9
        print("W=%d fwd rows=%d seg=%d  r04 plain+pack %.4f ms  r05 chunked %.4f ms  "
              "(%.0f -> %.0f GB/s algorithmic)" % (W, rw, cw, t4, t5, gb / t4 * 1e3, gb / t5 * 1e3))

        def r04_rev():
            return T.fwt_reverse(s4.permute(1, 0, 2).reshape(rw, C), w, lev, ctx)

        def r05_rev():
            return T.fwt_chunks_to_rows(s4, w, lev, ctx)

        assert torch.equal(r04_rev(), r05_rev()), "reverse forms differ"
        t4, t5 = med_ms(r04_rev, reps), med_ms(r05_rev, reps)
        print("W=%d rev rows=%d seg=%d  r04 unpack+plain %.4f ms  r05 chunked %.4f ms  "
              "(%.0f -> %.0f GB/s algorithmic)" % (W, rw, cw, t4, t5, gb / t4 * 1e3, gb / t5 * 1e3))
    print("forms identical at every W (torch.equal)")


if __name__ == "__main__":
    main()

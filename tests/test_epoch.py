"""The fused forward tail's arrival counter (jwave_amd/csrc/jwv_epoch.hpp):
the counter is never reset, each launch is told the value its last arriver
reads.  CPU test: the header is compiled with g++ and driven through launches
whose blocks arrive in a random order, across the 2^32 wrap, and through a
launch that dies part-way followed by the host's resync (capi.cpp
tail_resync: counter and base zeroed together)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "jwave_amd", "csrc")

PROG = r"""
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
#include "jwv_epoch.hpp"
using namespace jwv;
static std::mt19937 rng(7);
// one launch of nU blocks: returns how many blocks saw themselves as last,
// and which arrival position that was; `die_after` < nU stops it part-way
static int launch(uint32_t& counter, uint32_t base, uint32_t nU, uint32_t die_after, int* pos) {
  const uint32_t target = tail_last_old(base, nU);
  int lasts = 0;
  for (uint32_t k = 0; k < nU && k < die_after; ++k) {
    const uint32_t old = counter++;          // the block's atomic add
    if (old == target) { ++lasts; *pos = (int)k; }
  }
  return lasts;
}
int main() {
  const uint32_t starts[] = {0u, 12345u, 0xFFFFFFF0u, 0xFFFFFFFFu};
  for (uint32_t s : starts) {
    uint32_t counter = s, base = s;
    for (int call = 0; call < 200; ++call) {
      const uint32_t nU = 1 + rng() % 300;
      int pos = -1;
      if (launch(counter, base, nU, nU, &pos) != 1 || pos != (int)nU - 1) {
        std::printf("FAIL start=%u call=%d nU=%u pos=%d\n", s, call, nU, pos); return 1;
      }
      base = tail_next_base(base, nU);
      if (base != counter) { std::printf("FAIL base drift\n"); return 1; }
    }
  }
  // a launch that dies part-way: without the resync the next launch's last
  // arriver is missed; with it (counter = base = 0) the next launch is right
  {
    uint32_t counter = 0, base = 0; int pos = -1;
    launch(counter, base, 64, 20, &pos);
    int bad = launch(counter, tail_next_base(base, 64), 64, 64, &pos);
    if (bad != 0) { std::printf("FAIL expected a missed last arriver without resync\n"); return 1; }
    counter = 0; base = 0;  // tail_resync
    if (launch(counter, base, 64, 64, &pos) != 1 || pos != 63) { std::printf("FAIL after resync\n"); return 1; }
  }
  std::printf("ok\n");
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_tail_epoch_arithmetic(tmp_path):
    src = tmp_path / "epoch.cpp"
    exe = tmp_path / "epoch"
    src.write_text(PROG)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", HDR, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr

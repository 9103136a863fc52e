"""Multi-process tests of the sharded paths:
world sizes 2 and 3 with the gloo backend on CPU; every rank's compute is the
oracle, and the gathered result must equal the single-process oracle result
bit for bit (batch blocks, 2-D all-to-all transpose, MODWT ring halos)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from jwave_amd import distributed as D  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, backend="gloo", timeout=300):
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                               "--rank", str(r), "--world", str(world), "--port", str(port),
                               "--backend", backend],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out.decode(errors="replace")))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-4000:]
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_paths_gloo(world):
    outs = _launch(world)
    assert all("OK" in o for _, o in outs)


def test_shard_range_covers():
    for total in (0, 1, 7, 8, 4096, 10_000_000):
        for W in (1, 2, 3, 8):
            spans = [D.shard_range(total, W, r) for r in range(W)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_modwt_halo():
    # (L-1)(2^J - 1): Daubechies4 (L=8) J=8 -> 1785
    assert D.modwt_halo(8, 8) == 1785
    assert D.modwt_halo(2, 1) == 1


def test_2d_shape_check():
    with pytest.raises(ValueError):
        D._check_2d(64, 100, 3)


@pytest.mark.gpu
def test_sharded_paths_nccl_single_rank():
    """World size 1 over RCCL on the box's one GPU: the HIP backend through the
    same code (exchanges degenerate to local copies)."""
    if torch.cuda.device_count() < 1:
        pytest.fail("no GPU")
    outs = _launch(1, backend="nccl")
    assert "OK" in outs[0][1]

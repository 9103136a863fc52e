"""Host-side checks of the in-place reverse window layout (fwt1_kernels.hpp,
Rev1Geo::ip_doff / ip_fits; used by fwt_rev_tile1 and fwt_rev_tile16).

LDS holds [a_K | d_{K-1} | ... | d_0]; level l reads its approximations at 0
and its details at ip_doff(l), and writes its len(l) outputs over [0, len(l))
after a barrier.  The kernel relies on:
  * no level's outputs reach a detail window a later level still reads
    (len(l) <= ip_doff(l-1)), asserted at compile time for the compiled
    geometries and restated here for every bank and tile the planner can pick;
  * each level's reads stay inside its windows plus the 4-double pad (a
    couple reads up to 3 values past its window);
  * the layout is smaller than the ping-pong one, which is the point.
"""
import pytest


def c(l, L):
    q = L // 2
    cc = 0
    for _ in range(l):
        cc = ((cc // 2 + (q - 1)) + 1) & ~1
    return cc


def length(l, L, T):
    return (T >> l) + c(l, L)


def ip_doff(l, L, T, K):
    o = length(K, L, T)
    for k in range(K - 1, l, -1):
        o += length(k + 1, L, T)
    return o


def ip_lds(L, T, K):
    return ip_doff(-1, L, T, K) + 4


def pingpong_lds(L, T, K):
    dtotal = sum(length(k + 1, L, T) for k in range(K))
    return dtotal + length(1, L, T) + (max(length(2, L, T), length(K, L, T)) if K >= 2 else 0) + 4


GEOS = [(L, T, K) for L in (2, 4, 6, 8, 10, 12, 14, 16, 20, 24, 32)
        for T in (256, 512, 1024, 2048, 4096, 8192) for K in range(1, 8)
        if (T >> K) >= 2 and ((T >> K) & 1) == 0]


@pytest.mark.parametrize("L,T,K", GEOS)
def test_outputs_never_reach_unread_windows(L, T, K):
    for l in range(1, K):
        assert length(l, L, T) <= ip_doff(l - 1, L, T, K)


@pytest.mark.parametrize("L,T,K", GEOS)
def test_reads_stay_in_windows_plus_pad(L, T, K):
    total = ip_lds(L, T, K)
    for l in range(K):
        # details of level l: len(l+1) values at ip_doff(l), + up to 3 past
        assert ip_doff(l, L, T, K) + length(l + 1, L, T) + 3 < total
        # approximations at 0: len(l+1) values; the over-read lands on other
        # (stale or unread) windows inside the allocation, never outside it
        assert length(l + 1, L, T) + 3 < total


@pytest.mark.parametrize("L,T,K,rows,b_ip,b_pp", [
    (16, 2048, 3, 1, 16800, 27088),   # config-3 rows: 27 -> 17 kB
    (16, 256, 3, 16, 39424, 60672),   # 16-column slabs: 61 -> 39 kB
])
def test_config3_lds_budget(L, T, K, rows, b_ip, b_pp):
    assert rows * ip_lds(L, T, K) * 8 == b_ip
    assert rows * pingpong_lds(L, T, K) * 8 == b_pp
    # blocks per CU by LDS (160 KiB): the in-place layout's reason to exist
    assert 163840 // b_ip > 163840 // b_pp

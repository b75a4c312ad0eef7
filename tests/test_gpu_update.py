"""GPU parity for the incremental-update entry points against the oracle:
click_update_in_cksum (include/clicknet/ip.h:177-185) and
click_update_zero_in_cksum (ip.h:196-201, lib/in_cksum.c:113-121), at odd
and even offsets, with all-zero payloads that need the fixup, and fields
past the packet end (domain guard: nothing written)."""
import ctypes

import numpy as np
import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def ctx(torch):
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def make(rng, n):
    """Packets at arbitrary offsets: random bytes, or all zero with a
    stored checksum 0xFFFF (an all-zero ICMP message) at sum_off 2."""
    lens = rng.integers(0, 80, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 5))
        off[i] = pos
        pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    for i in range(n):
        if rng.random() < 0.3:
            o, L = int(off[i]), int(lens[i])
            arena[o:o + L] = 0
            if L >= 4:
                arena[o + 2:o + 4] = 0xFF
    return arena, off, lens


def oracle_update(arena, off, lens, sum_off, hw_off, new_hw, zero_fix, zero_lo, replace=True):
    L = oracle_lib.load_oracle()
    n = len(off)
    st = np.zeros(n, np.uint8)
    sums = np.zeros(n, np.uint16)
    for i in range(n):
        o, ln = int(off[i]), int(lens[i])
        if sum_off + 2 > ln or (replace and hw_off + 2 > ln):
            st[i] = 1
            continue
        p = arena[o:o + ln]
        csum = int(p[sum_off:sum_off + 2].view(np.uint16)[0])
        if replace:
            old = int(p[hw_off:hw_off + 2].view(np.uint16)[0])
            p[hw_off:hw_off + 2] = np.array([new_hw[i]], np.uint16).view(np.uint8)
            csum = L.oracle_update_in_cksum(csum, old, int(new_hw[i]))
            p[sum_off:sum_off + 2] = np.array([csum], np.uint16).view(np.uint8)
        if zero_fix and csum == 0:
            z = p[zero_lo:].tobytes()
            fixed = L.oracle_update_zero_in_cksum(csum, z, len(z))
            if fixed != csum:
                csum = fixed
                p[sum_off:sum_off + 2] = np.array([csum], np.uint16).view(np.uint8)
                st[i] = 2
        sums[i] = csum
    return st, sums


@pytest.mark.parametrize("sum_off,hw_off,zero_lo", [(2, 0, 0), (10, 8, 0), (6, 0, 0), (3, 11, 1)])
@pytest.mark.parametrize("zero_fix", [True, False])
def test_update_in_cksum(torch, ctx, sum_off, hw_off, zero_lo, zero_fix):
    import click_amd
    rng = np.random.default_rng(sum_off * 31 + hw_off + 7 * zero_fix)
    n = 3000
    arena, off, lens = make(rng, n)
    new_hw = rng.integers(0, 65536, n).astype(np.uint16)
    new_hw[rng.random(n) < 0.4] = 0                  # keeps all-zero packets zero: the fixup case
    ref = arena.copy()
    st_r, sums_r = oracle_update(ref, off, lens, sum_off, hw_off, new_hw, zero_fix, zero_lo)
    a = torch.from_numpy(arena).cuda()
    b = click_amd.Batch(a, n, off=torch.from_numpy(off.view(np.int64)).cuda(),
                        length=torch.from_numpy(lens.view(np.int32)).cuda())
    st, sums = ctx.update_in_cksum(b, sum_off, hw_off, torch.from_numpy(new_hw.view(np.int16)).cuda(),
                                   zero_fix=zero_fix, zero_lo=zero_lo)
    assert np.array_equal(st.cpu().numpy(), st_r)
    assert np.array_equal(sums.cpu().numpy().view(np.uint16), sums_r)
    assert np.array_equal(a.cpu().numpy(), ref)
    if zero_fix and sum_off == 2:
        assert (st_r == 2).sum() > 0                 # the fixup ran


def test_update_zero_in_cksum(torch, ctx):
    import click_amd
    rng = np.random.default_rng(99)
    n = 4000
    arena, off, lens = make(rng, n)
    for i in range(n):                               # zero checksums over zero and nonzero data
        o, L = int(off[i]), int(lens[i])
        if L >= 4 and rng.random() < 0.5:
            arena[o + 2:o + 4] = 0
    ref = arena.copy()
    st_r, sums_r = oracle_update(ref, off, lens, 2, 0, None, True, 0, replace=False)
    a = torch.from_numpy(arena).cuda()
    b = click_amd.Batch(a, n, off=torch.from_numpy(off.view(np.int64)).cuda(),
                        length=torch.from_numpy(lens.view(np.int32)).cuda())
    st, sums = ctx.update_zero_in_cksum(b, 2, 0)
    assert np.array_equal(st.cpu().numpy(), st_r)
    assert np.array_equal(sums.cpu().numpy().view(np.uint16), sums_r)
    assert np.array_equal(a.cpu().numpy(), ref)
    assert (st_r == 2).sum() > 0 and (st_r == 0).sum() > 0 and (st_r == 1).sum() > 0

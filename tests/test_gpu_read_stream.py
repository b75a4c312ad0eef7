"""The read-ceiling probe (clk_read_stream, every CLK_TUNE_READ_SHAPE): each
shape must read every 16 B chunk of the buffer exactly once -- including the
tails past its last whole step -- or the ceiling `bench.py` reports would be
a rate over bytes not read.  Each lane adds the xor of its chunks' four words
into a u32, so the u64 the kernel accumulates equals, mod 2^32, the sum of
every chunk's xor over the buffer whatever the shape's partition."""
import numpy as np
import pytest

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


@pytest.mark.parametrize("shape", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("chunks", [1, 37, 16 * 96 * 16, 3 * 16 * 96 * 16 + 1001, (1 << 22) + 12345])
def test_read_stream_reads_every_chunk_once(ctx, torch, shape, chunks):
    rng = np.random.default_rng(chunks * 7 + shape)
    host = rng.integers(0, 2 ** 32, size=(chunks, 4), dtype=np.uint64).astype(np.uint32)
    x = host[:, 0] ^ host[:, 1] ^ host[:, 2] ^ host[:, 3]
    want = int(x.astype(np.uint64).sum()) & 0xFFFFFFFF
    buf = torch.from_numpy(host.reshape(-1).view(np.uint8).copy()).cuda()
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.tune(read_shape=shape)
    try:
        ctx.read_stream(buf, out=out)
        torch.cuda.synchronize()
    finally:
        ctx.tune(read_shape=0)
    assert int(out.item()) & 0xFFFFFFFF == want


def test_read_shape_out_of_range(ctx):
    from click_amd import ClickAmdError
    with pytest.raises(ClickAmdError):
        ctx.tune(read_shape=6)

"""OCP-MX quantisation (ops/mx.py): packing round trips, exact representability, block exponents,
and the CPU quantise-then-multiply semantics of MXWeight (the oracle of the gfx950 kernel test,
tests/test_mx_gemm_gpu.py)."""
import pytest
import torch

from shuffle_exchange_amd.ops import mx


@pytest.mark.parametrize("fmt", list(mx.FORMATS))
def test_pack_roundtrip(fmt):
    bits = mx.FORMATS[fmt][3]
    g = torch.Generator().manual_seed(0)
    codes = torch.randint(0, 1 << bits, (5, 64), generator=g)
    if bits == 8:
        codes = torch.where((codes & 0x7F) == 0x7F, codes - 1, codes)  # no e4m3 NaN
    p = mx.pack(codes, bits)
    assert p.shape == (5, 64 * bits // 8) and p.dtype == torch.uint8
    assert torch.equal(mx.unpack(p, bits, 64), codes)


def test_fp6_bit_order():
    # element j at bits [6j, 6j+6) of the little-endian byte stream
    codes = torch.zeros(1, 4, dtype=torch.int64)
    codes[0, 1] = 0x3F
    p = mx.pack(codes, 6)
    assert p.tolist() == [[0xC0, 0x0F, 0x00]]


@pytest.mark.parametrize("fmt", list(mx.FORMATS))
def test_representable_values_are_exact(fmt):
    _, eb, mb, bits, fmax = mx.FORMATS[fmt]
    if bits == 8:
        vals = torch.arange(0, 0x7F, dtype=torch.int64).to(torch.uint8).view(torch.float8_e4m3fn).float()
    else:
        vals = mx._values(eb, mb)
    assert float(vals.max()) == fmax
    # one block = the largest value (exponent 0) + representable values, both signs
    row = torch.cat([vals, -vals])[:32]
    row[0] = fmax
    x = row.repeat(2, 4)
    q, s = mx.quantize(x, fmt)
    assert torch.all(s == 127)
    assert torch.equal(mx.dequantize(q, s, fmt, x.shape[1]), x)


@pytest.mark.parametrize("fmt", list(mx.FORMATS))
def test_block_exponent_and_error(fmt):
    fmax = mx.FORMATS[fmt][4]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 256, generator=g) * torch.logspace(-3, 3, 8)[:, None]
    q, s = mx.quantize(x, fmt)
    blocks = x.reshape(8, -1, 32).abs().amax(-1)
    e = s.float() - 127
    assert torch.all(blocks * torch.exp2(-e) <= fmax)       # nothing saturates
    assert torch.all(blocks * torch.exp2(-(e - 1)) > fmax)   # and the exponent is the smallest such
    d = mx.dequantize(q, s, fmt, 256)
    rel = ((d - x).abs() / blocks.repeat_interleave(32, 1)).max()
    # error <= half the largest code gap (x 2^e), and the block max is >= fmax / 2 (x 2^e)
    if fmt == "mxfp8":
        vals = torch.arange(0, 0x7F, dtype=torch.int64).to(torch.uint8).view(torch.float8_e4m3fn).float()
    else:
        vals = mx._values(*mx.FORMATS[fmt][1:3])
    bound = (vals.sort().values.diff().max() / 2) / (fmax / 2)
    assert rel <= bound * 1.0001


def test_mxweight_cpu_semantics():
    torch.manual_seed(0)
    w = torch.randn(256, 384) * 0.05
    x = torch.randn(7, 384)
    b = torch.randn(256)
    for fmt in mx.FORMATS:
        W = mx.MXWeight(w, fmt)
        y = W.linear(x.to(torch.bfloat16), bias=b)
        xq, xs = mx.quantize(x.to(torch.bfloat16).float(), "mxfp8")
        ref = mx.dequantize(xq, xs, "mxfp8", 384) @ W.dequantize(torch.float32).t() + b
        torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
        # and the quantised product is a faithful approximation of the full-precision one
        rel = (y.float() - (x @ w.t() + b)).norm() / (x @ w.t() + b).norm()
        assert rel < {"mxfp8": 0.05, "mxfp6": 0.1, "mxfp6_e2m3": 0.1, "mxfp4": 0.25}[fmt]
    assert mx.MXWeight(w, "mxfp4").nbytes == 256 * 384 // 2 + 256 * 384 // 32

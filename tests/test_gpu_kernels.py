"""Numerics of the HIP/CDNA4 streaming kernels (csrc/hip/hbm_probe.hip) on a
real MI355X: each kernel runs on torch device tensors and its output is
compared with a plain PyTorch reference of the same op (fp32 for triad,
bit-exact for copy/write). Every unroll x cache-policy x workgroups-per-CU
variant is covered, with sizes that exercise the grid-stride tail loops."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch  # first: the probe library then binds to torch's HIP runtime

    assert torch.cuda.is_available()
    torch.cuda.init()
    from flex_gpu_scheduler_amd.ops.hip_probe import HipProbe

    return torch, HipProbe()


# 1 MiB + 48 B: not a multiple of (blocks x 256 lanes x unroll), so every
# variant runs its remainder loop.
ODD = (1 << 20) + 48
VARIANTS = [(u, nt, b) for u in (1, 4, 8) for nt in (True, False) for b in (4, 8, 16)]


def _pattern(torch, n_vec4: int, seed: int):
    s = seed & 0xFFFFFFFF
    lane = [s, s ^ 0x55555555, (s + 1) & 0xFFFFFFFF, ~s & 0xFFFFFFFF]
    lane = [v - (1 << 32) if v >= (1 << 31) else v for v in lane]  # as int32 bit patterns
    return torch.tensor(lane, dtype=torch.int32, device="cuda").repeat(n_vec4)


@pytest.mark.parametrize("nbytes", [16, 4096, ODD, 64 << 20])
def test_copy_is_bit_exact(env, nbytes):
    torch, pr = env
    src = torch.randint(-(1 << 31), (1 << 31) - 1, (nbytes // 4,), dtype=torch.int32, device="cuda")
    dst = torch.zeros_like(src)
    pr.copy(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)


@pytest.mark.parametrize("u,nt,bpc", VARIANTS)
def test_copy_variants(env, u, nt, bpc):
    torch, pr = env
    src = torch.randint(-(1 << 31), (1 << 31) - 1, (ODD // 4,), dtype=torch.int32, device="cuda")
    dst = torch.full_like(src, -1)
    pr.copy(dst, src, variant=pr.variant(u, nt, bpc))
    assert torch.equal(dst, src)


@pytest.mark.parametrize("seed", [7, 0, 0xDEADBEEF])
@pytest.mark.parametrize("u,nt,bpc", [(1, False, 4), (4, True, 8), (8, True, 16)])
def test_write_pattern(env, seed, u, nt, bpc):
    torch, pr = env
    dst = torch.zeros(ODD // 4, dtype=torch.int32, device="cuda")
    pr.write_pattern(dst, seed=seed, variant=pr.variant(u, nt, bpc))
    assert torch.equal(dst, _pattern(torch, ODD // 16, seed))


@pytest.mark.parametrize("nbytes", [4096, ODD, 256 << 20])
@pytest.mark.parametrize("scale", [3.0, -0.5])
def test_triad_matches_fp32_reference(env, nbytes, scale):
    torch, pr = env
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    b = torch.randn(nbytes // 4, dtype=torch.float32, device="cuda", generator=g)
    c = torch.randn(nbytes // 4, dtype=torch.float32, device="cuda", generator=g)
    a = torch.full_like(b, float("nan"))
    pr.triad(a, b, c, scale=scale)
    ref = b + scale * c  # plain PyTorch fp32
    # The kernel may contract x + s*y into one FMA (one rounding instead of
    # two): allow 1 ulp of the operands' magnitude, nothing more.
    torch.testing.assert_close(a, ref, rtol=2.4e-7, atol=2.4e-7 * (1 + abs(scale)) * 8)
    assert not torch.isnan(a).any()


@pytest.mark.parametrize("u,nt,bpc", VARIANTS)
def test_triad_variants(env, u, nt, bpc):
    torch, pr = env
    b = torch.arange(ODD // 4, dtype=torch.float32, device="cuda")
    c = torch.full_like(b, 0.25)
    a = torch.zeros_like(b)
    pr.triad(a, b, c, scale=4.0, variant=pr.variant(u, nt, bpc))
    assert torch.equal(a, b + 1.0)  # exact in fp32 for these values


@pytest.mark.parametrize("mask", [0x01, 0x0F, 0xFF])
def test_xcd_pinned_copy_and_write(env, mask):
    torch, pr = env
    from flex_gpu_scheduler_amd.ops.hip_probe import probe as _  # noqa: F401 - same library

    if pr.xcd_census(0, 2048)["distinct_xcds"] < 8 and mask != 0x01:
        pytest.skip("device is partitioned")
    src = torch.randint(-(1 << 31), (1 << 31) - 1, ((8 << 20) // 4 + 12,), dtype=torch.int32, device="cuda")
    dst = torch.zeros_like(src)
    pr.pinned(dst, src, xcd_mask=mask)
    assert torch.equal(dst, src)
    pr.pinned(dst, None, xcd_mask=mask)
    assert torch.equal(dst, torch.tensor([1, 2, 3, 4], dtype=torch.int32, device="cuda").repeat(src.numel() // 4))


def test_rejects_misaligned_and_host_buffers(env):
    torch, pr = env
    x = torch.zeros(64, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        pr.copy(x[1:17], x[20:36])  # 4-byte offset
    with pytest.raises(ValueError):
        pr.copy(torch.zeros(16, dtype=torch.int32), torch.zeros(16, dtype=torch.int32))

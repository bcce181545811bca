"""T1: HIP kernel <-> fp32 PyTorch reference parity.

Every hand-written gfx950 kernel is compared against a plain fp32 PyTorch
implementation of the same op.  bf16 operands -> tolerances scale with K.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module")
def K():
    from iit_amd.ops import hip_kernels
    hip_kernels.lib()
    return hip_kernels


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,Kd", [(256, 384, 256), (4096, 768, 768), (200, 130, 72), (64, 50257 // 7, 64)])
def test_gemm_nn_bias(K, M, N, Kd):
    torch.manual_seed(0)
    A = torch.randn(M, Kd, device=dev)
    W = torch.randn(N, Kd, device=dev) / math.sqrt(Kd)  # [N][K]
    b = torch.randn(N, device=dev)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    K.gemm(bf(A), bf(W), C, M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, epi=K.EPI_BF16, bias0=b)
    ref = bf(A).float() @ bf(W).float().T + b
    assert rel_err(C, ref) < 1e-2


def test_gemm_asymmetric_identity(K):
    """A = I with an asymmetric B catches row/col swaps in the C layout."""
    n = 128
    A = torch.eye(n, device=dev)
    B = torch.arange(n * n, device=dev, dtype=torch.float32).view(n, n) % 97
    C = torch.empty(n, n, dtype=torch.float32, device=dev)
    K.gemm(bf(A), bf(B), C, M=n, N=n, K=n, lda=n, ldb=n, ldc=n, epi=K.EPI_F32_STORE)
    # C = A @ B^T with B stored [N][K]
    assert torch.equal(C, bf(B).float().T)


@pytest.mark.parametrize("M,N,T", [(768, 768, 4096), (64, 200, 96), (128, 256, 300)])
def test_gemm_kmajor_accumulate(K, M, N, T):
    torch.manual_seed(1)
    X = torch.randn(T, M, device=dev)
    G = torch.randn(T, N, device=dev)
    out = torch.randn(M, N, device=dev)
    ref = out + bf(X).float().T @ bf(G).float()
    K.gemm(bf(X), bf(G), out, M=M, N=N, K=T, lda=M, ldb=N, ldc=N, mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_ACC)
    assert rel_err(out, ref) < 1e-2


def test_gemm_kmajor_fp32_b_splitk(K):
    torch.manual_seed(2)
    M, N, T = 256, 128, 8192
    X = torch.randn(T, M, device=dev)
    G = torch.randn(T, N, device=dev)
    out = torch.zeros(M, N, device=dev)
    K.gemm(bf(X), G, out, M=M, N=N, K=T, lda=M, ldb=N, ldc=N, mode=K.MODE_AKM | K.MODE_BKM | K.MODE_BF32,
           epi=K.EPI_F32_ACC, splits=4)
    ref = bf(X).float().T @ bf(G).float()
    assert rel_err(out, ref) < 1e-2


def test_gemm_fp32_a_residual_gelu(K):
    torch.manual_seed(3)
    M, N, Kd = 512, 256, 192
    A = torch.randn(M, Kd, device=dev)
    W = torch.randn(N, Kd, device=dev) / math.sqrt(Kd)
    b = torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev)
    C = torch.empty(M, N, device=dev)
    K.gemm(A, bf(W), C, M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, mode=K.MODE_AF32, epi=K.EPI_F32_STORE)
    assert rel_err(C, bf(A).float() @ bf(W).float().T) < 1e-2
    K.gemm(bf(A), bf(W), C, M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, epi=K.EPI_F32_RESID, bias0=b, resid=R, ldr=N)
    assert rel_err(C, R + bf(A).float() @ bf(W).float().T + b) < 1e-2
    post = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    K.gemm(bf(A), bf(W), post, C2=pre, M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, ldc2=N, epi=K.EPI_GELU, bias0=b)
    from iit_amd.ops.torch_ops import gelu_new
    ref_pre = bf(A).float() @ bf(W).float().T + b
    assert rel_err(pre, ref_pre) < 1e-2
    assert rel_err(post, gelu_new(ref_pre)) < 1e-2


@pytest.mark.parametrize("d,affine,bf16_dy", [(768, False, False), (768, True, True), (130, True, False), (1024, True, False), (256, True, True),
                                              (4096, False, True), (66, False, False)])
def test_layernorm(K, d, affine, bf16_dy):
    """Vector (d % 4 == 0) and scalar kernels; affine dw/db reduction; fused skip gradient + bf16 twin."""
    torch.manual_seed(4)
    T = 1000
    x = torch.randn(T, d, device=dev) * 3 + 1
    w = torch.randn(d, device=dev) if affine else None
    b = torch.randn(d, device=dev) if affine else None
    y = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    mean = torch.empty(T, device=dev)
    rstd = torch.empty(T, device=dev)
    K.ln_fwd(x, w, b, y, mean, rstd, T, d, 1e-5)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True) if affine else None
    br = b.clone().requires_grad_(True) if affine else None
    ref = torch.nn.functional.layer_norm(xr, (d,), wr, br, 1e-5)
    assert rel_err(y, ref) < 1e-2
    g = torch.randn(T, d, device=dev)
    if bf16_dy:
        g = bf(g)
    ref.backward(g.float())
    dres = torch.randn(T, d, device=dev)
    dx = torch.empty(T, d, device=dev)
    dx16 = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    # the affine gradients accumulate into the existing slots (fused into the dx pass for d <= 1024, iit_ln_bwd_part)
    dw = torch.ones(d, device=dev) if affine else None
    db = torch.ones(d, device=dev) if affine else None
    K.ln_bwd(g, x, mean, rstd, w, dx, dw, db, T, d, dres=dres, dx16=dx16)
    assert rel_err(dx, xr.grad + dres) < 1e-3
    assert torch.equal(dx16, dx.to(torch.bfloat16))
    if affine:
        assert rel_err(dw - 1, wr.grad) < 1e-4 and rel_err(db - 1, br.grad) < 1e-4
    elif d % 4 == 0:  # LNPre backward from the bf16 output (xhat) instead of the fp32 input
        dxh = torch.empty(T, d, device=dev)
        K.ln_bwd_xh16(g, y, rstd, dxh, T, d, dres=dres, dx16=dx16)
        assert rel_err(dxh, xr.grad + dres) < 1e-2
        assert torch.equal(dx16, dxh.to(torch.bfloat16))


def test_gelu_fwd_and_pos_bwd(K):
    from iit_amd.ops.torch_ops import gelu_new
    torch.manual_seed(12)
    pre = bf(torch.randn(300, 1032, device=dev) * 3)
    out = torch.empty(300, 1040, dtype=torch.bfloat16, device=dev)[:, :1024]
    K.gelu_fwd(pre[:, :1024], out, 300, 1024)
    assert rel_err(out, gelu_new(pre[:, :1024].float())) < 4e-3
    out2 = torch.empty(300, 7, dtype=torch.bfloat16, device=dev)
    K.gelu_fwd(pre[:, :7], out2, 300, 7)  # scalar path
    assert rel_err(out2, gelu_new(pre[:, :7].float())) < 4e-3
    K.gelu_fwd(pre[:, :1024], out, 300, 1024, erf=True)
    assert rel_err(out, torch.nn.functional.gelu(pre[:, :1024].float())) < 4e-3
    g = bf(torch.randn(300, 1024, device=dev))
    x = pre[:, :1024].float().contiguous().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(g.float())
    dpre = torch.empty(300, 1024, dtype=torch.bfloat16, device=dev)
    K.dgelu(g, pre[:, :1024].contiguous(), dpre, erf=True)
    assert rel_err(dpre, x.grad) < 1e-2
    B, S, d = 33, 16, 768
    g = torch.randn(B * S, d, device=dev)
    tok = torch.randint(0, 50, (B * S,), device=dev)
    dWE = torch.zeros(50, d, device=dev)
    dWpos = torch.randn(S + 3, d, device=dev)
    ref_pos = dWpos.clone()
    ref_pos[:S] += g.view(B, S, d).sum(0)
    K.embed_pos_bwd(tok, g, dWE, dWpos, B, S, d)
    assert torch.allclose(dWpos, ref_pos, atol=1e-4, rtol=1e-4)
    assert torch.allclose(dWE, torch.zeros(50, d, device=dev).index_add_(0, tok, g), atol=1e-4)


@pytest.mark.parametrize("S,H,dh,causal", [(16, 12, 64, True), (16, 4, 16, True), (33, 3, 32, True), (5, 12, 64, True),
                                           (11, 3, 32, True), (16, 2, 128, True), (13, 5, 96, False),
                                           (16, 12, 64, False), (40, 4, 64, False)])
def test_attention_fwd_bwd_with_head_splice(K, S, H, dh, causal):
    """S <= 16 with dh in {32,64,96,128} runs the MFMA kernel (csrc/attn_mfma.hip); the rest the VALU one."""
    torch.manual_seed(5)
    B = 7
    qkv = torch.randn(B, S, 3, H, dh, device=dev)
    zsrc = torch.randn(B, S, H, dh, device=dev)
    patched = [1] if H > 1 else []
    mask = K.heads_to_mask(patched)
    z = torch.empty(B, S, H, dh, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H * S, device=dev)
    q16 = bf(qkv).contiguous()
    K.attn_small_fwd(q16, z, lse, bf(zsrc), mask, B, S, H, dh, 3 * H * dh, H * dh, H * dh, 1 / math.sqrt(dh), causal)
    qf = q16.float().requires_grad_(True)
    q, k, v = qf[:, :, 0], qf[:, :, 1], qf[:, :, 2]
    sc = torch.einsum("bqhe,bkhe->bhqk", q, k) / math.sqrt(dh)
    if causal:
        sc = sc.masked_fill(~torch.ones(S, S, dtype=torch.bool, device=dev).tril(), float("-inf"))
    ref_lse = sc.logsumexp(-1)  # [B,H,S]
    ref = torch.einsum("bkhe,bhqk->bqhe", v, sc.softmax(-1))
    live = [h for h in range(H) if h not in patched]
    assert torch.allclose(lse.view(B, H, S)[:, live], ref_lse[:, live].detach(), atol=2e-2, rtol=1e-2)
    for h in patched:
        ref = ref.clone()
        ref[:, :, h] = bf(zsrc)[:, :, h].float()
    assert rel_err(z, ref) < 1e-2
    g = torch.randn(B, S, H, dh, device=dev)
    ref.backward(g)
    dq = torch.empty_like(q16)
    K.attn_small_bwd(q16, bf(g), lse, dq, mask, B, S, H, dh, 3 * H * dh, H * dh, 1 / math.sqrt(dh), causal)
    assert rel_err(dq, qf.grad) < 2e-2
    for i in range(3):  # q, k and v gradients separately
        assert rel_err(dq[:, :, i], qf.grad[:, :, i]) < 2e-2
    for h in patched:
        assert dq[:, :, :, h].abs().max().item() == 0


def test_cross_entropy(K):
    torch.manual_seed(6)
    R, V = 64, 50257
    from iit_amd.ops.hip_ops import cross_entropy
    logits = (torch.randn(R, V, device=dev) * 4).requires_grad_(True)
    labels = torch.randint(0, V, (R,), device=dev)
    loss = cross_entropy(logits, labels) * 0.7
    loss.backward()
    lr = logits.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, labels) * 0.7
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4
    assert rel_err(logits.grad, lr.grad) < 1e-4


def test_flat_adam_matches_torch(K):
    torch.manual_seed(7)
    from iit_amd.engine.flat import FlatParams
    from iit_amd.ops.optim import FusedAdam
    m1 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 33)).to(dev)
    m2 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 33)).to(dev)
    m2.load_state_dict(m1.state_dict())
    flat = FlatParams(m1)
    opt1 = FusedAdam(flat, lr=1e-2)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-2)
    for _ in range(5):
        x = torch.randn(16, 64, device=dev)
        opt1.zero_grad()
        m1(x).pow(2).sum().backward()
        opt1.step(clip_norm=1.0)
        opt2.zero_grad()
        m2(x).pow(2).sum().backward()
        torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
        opt2.step()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, atol=1e-5, rtol=1e-4)


def test_flat_adam_row_restriction_is_exact(K):
    """Skipping embedding rows that never get gradient leaves the update identical to the full pass (up to the
    summation order of the clip norm's partial sums, which follow the span table)."""
    torch.manual_seed(13)
    from iit_amd.engine.flat import FlatParams
    from iit_amd.ops.optim import FusedAdam

    def make():
        torch.manual_seed(13)
        return torch.nn.ModuleDict({"emb": torch.nn.Embedding(5000, 64), "lin": torch.nn.Linear(64, 7)}).to(dev)

    m1, m2 = make(), make()
    f1, f2 = FlatParams(m1, with_bf16_shadow=True), FlatParams(m2, with_bf16_shadow=True)
    live = torch.tensor([3, 4, 5, 900, 4999, 17])
    assert f1.restrict_rows(m1["emb"].weight, live)
    o1, o2 = FusedAdam(f1, lr=1e-2), FusedAdam(f2, lr=1e-2)
    for _ in range(4):
        idx = live[torch.randint(0, len(live), (32,))].to(dev)
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            m["lin"](m["emb"](idx)).pow(2).sum().backward()
            o.step(clip_norm=1.0)
    assert f1._inactive, "restriction must survive the first-step validation"
    assert torch.allclose(f1.data, f2.data, rtol=1e-5, atol=1e-7)
    assert torch.allclose(o1.exp_avg, o2.exp_avg, rtol=1e-4, atol=1e-6)
    off = f1.offset_of(m1["emb"].weight)
    dead = torch.ones(5000, dtype=torch.bool)
    dead[live] = False
    w1 = f1.data[off:off + 5000 * 64].view(5000, 64)
    w2 = f2.data[off:off + 5000 * 64].view(5000, 64)
    assert torch.equal(w1[dead.to(dev)], w2[dead.to(dev)])  # untouched rows: bit-identical


def test_add_bf16_and_vector_dgelu(K):
    torch.manual_seed(8)
    M, N = 300, 768
    out = torch.randn(M, 800, device=dev)[:, :N]
    base = torch.randn(M, N, device=dev)
    y = torch.randn(M, N, device=dev).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    K.add_bf16(out, out.stride(0), base, N, y, N, b, M, N)
    assert torch.allclose(out, base + y.float() + b, atol=1e-6)
    acc = torch.randn(M, 770, device=dev)  # odd width -> scalar path
    ref = acc + torch.ones_like(acc)
    K.add_bf16(acc, 770, acc, 770, torch.ones(M, 770, device=dev, dtype=torch.bfloat16), 770, None, M, 770)
    assert torch.allclose(acc, ref)
    from iit_amd.ops.torch_ops import gelu_new
    pre = torch.randn(4096, 8, device=dev).to(torch.bfloat16)
    g = torch.randn(4096, 8, device=dev).to(torch.bfloat16)
    x = pre.float().requires_grad_(True)
    gelu_new(x).backward(g.float())
    out2 = torch.empty_like(pre)
    K.dgelu(g, pre, out2)
    assert rel_err(out2, x.grad) < 1e-2


def test_dispatch_blas16_epilogues(K):
    from iit_amd.ops import gemm_dispatch as gd
    torch.manual_seed(9)
    M, N, Kd = 512, 768, 1024
    A, W = bf(torch.randn(M, Kd, device=dev)), bf(torch.randn(N, Kd, device=dev) / 32)
    R, b = torch.randn(M, N, device=dev), torch.randn(N, device=dev)
    C = torch.empty(M, N, device=dev)
    gd._blas16(A, W, C, M, N, Kd, Kd, Kd, N, K.MODE_NN, K.EPI_F32_RESID, b, R, N)
    assert rel_err(C, R + A.float() @ W.float().T + b) < 1e-2
    G = torch.randn(Kd, N, device=dev)
    X, Y = bf(torch.randn(M, Kd, device=dev)), bf(torch.randn(M, N, device=dev))
    ref = G + X.float().T @ Y.float()
    gd._blas16(X, Y, G, Kd, N, M, Kd, N, N, K.MODE_AKM | K.MODE_BKM, K.EPI_F32_ACC, None, None, 0)
    assert rel_err(G, ref) < 1e-2


@pytest.mark.parametrize("T,N,f32", [(4096, 3072, False), (4096, 768, True), (300, 130, False), (77, 36, True)])
def test_colsum(K, T, N, f32):
    torch.manual_seed(10)
    x = torch.randn(T, N, device=dev)
    x = x if f32 else bf(x)
    out = torch.randn(N, device=dev)
    ref = out + x.float().sum(0)
    K.colsum_accum(x, N, out, T, N)
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3)


def test_cross_entropy_bf16_grad_kernel(K):
    torch.manual_seed(11)
    R, V = 8, 1000
    logits = torch.randn(R, V, device=dev) * 3
    labels = torch.randint(0, V, (R,), device=dev)
    loss = torch.empty(R, device=dev)
    lse = torch.empty(R, device=dev)
    amax = torch.empty(R, dtype=torch.long, device=dev)
    K.ce_fwd(logits, V, labels, loss, lse, amax, R, V)
    assert torch.allclose(lse, logits.logsumexp(-1), atol=1e-4)
    assert torch.equal(amax, logits.argmax(-1))
    out = torch.empty(R, 1008, dtype=torch.bfloat16, device=dev)
    g = torch.ones(1, device=dev)
    K.ce_bwd(logits, V, labels, lse, g, 1.0 / R, out, 1008, R, V)
    ref = (logits.softmax(-1) - torch.nn.functional.one_hot(labels, V)) / R
    assert rel_err(out[:, :V], ref) < 1e-2 and out[:, V:].abs().max() == 0


def test_cross_entropy_grad_bf16_twin(K):
    """ce_bwd with an fp32 output also writes the bf16 copy (same padded stride) the unembed GEMMs read."""
    torch.manual_seed(12)
    R, V = 8, 1000
    logits = torch.randn(R, V, device=dev) * 3
    labels = torch.randint(0, V, (R,), device=dev)
    loss, lse = torch.empty(R, device=dev), torch.empty(R, device=dev)
    K.ce_fwd(logits, V, labels, loss, lse, None, R, V)
    out = torch.full((R, 1008), 7.0, device=dev)
    out16 = torch.full((R, 1008), 7.0, dtype=torch.bfloat16, device=dev)
    K.ce_bwd(logits, V, labels, lse, torch.ones(1, device=dev), 1.0 / R, out, 1008, R, V, out16=out16)
    ref = (logits.softmax(-1) - torch.nn.functional.one_hot(labels, V)) / R
    assert rel_err(out[:, :V], ref) < 1e-5 and out[:, V:].abs().max() == 0
    assert torch.equal(out16, out.bfloat16())


def test_sumsq_2d_kernel(K):
    """gsq slots += sum of squares of a strided fp32 matrix (the fused-norm pass after a library GEMM)."""
    torch.manual_seed(13)
    c = torch.randn(300, 520, device=dev)
    gsq = torch.zeros(64, device=dev)
    K.sumsq_2d(c, 520, 300, 512, gsq)
    torch.testing.assert_close(gsq.sum(), c[:, :512].double().pow(2).sum().float(), rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("T,d,vocab", [(4096, 768, 40), (1000, 768, 5000), (130, 64, 3)])
def test_embed_bwd_repeated_tokens(K, T, d, vocab):
    """Embedding backward (atomic row adds, many repeated tokens) == index_add over the positions; W_pos too."""
    torch.manual_seed(T + vocab)
    S = 10 if T % 10 == 0 else 1
    B = T // S
    tok = torch.randint(0, vocab, (B, S), device=dev)
    g = torch.randn(B, S, d, device=dev)
    dWE = torch.randn(vocab, d, device=dev)
    dWpos = torch.randn(S, d, device=dev)
    ref_E = dWE.clone().index_add_(0, tok.reshape(-1), g.reshape(-1, d))
    ref_pos = dWpos + g.sum(0)
    K.embed_pos_bwd(tok, g, dWE, dWpos, B, S, d)
    torch.cuda.synchronize()
    torch.testing.assert_close(dWE, ref_E, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(dWpos, ref_pos, rtol=1e-5, atol=1e-4)


def test_embed_bwd_template_batches(K):
    """IOI-like batches (the same token at most positions across the batch, a few varied positions): the
    position-major embedding backward (runs of equal tokens summed in registers) == index_add."""
    torch.manual_seed(7)
    B, S, d, vocab = 256, 16, 768, 50257
    template = torch.randint(0, vocab, (S,), device=dev)
    tok = template.repeat(B, 1)
    for s in (2, 4, 9):
        tok[:, s] = torch.randint(0, 40, (B,), device=dev)
    g = torch.randn(B, S, d, device=dev)
    dWE = torch.zeros(vocab, d, device=dev)
    ref = torch.zeros(vocab, d, device=dev).index_add_(0, tok.reshape(-1), g.reshape(-1, d))
    K.embed_pos_bwd(tok, g, dWE, None, B, S, d)
    torch.cuda.synchronize()
    torch.testing.assert_close(dWE, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("n_ranges", [1, 64, 128, 129, 300])
def test_zero_ranges_many_ranges(K, n_ranges):
    """zero_ranges (the gradient arena's memset, up to 128 ranges per launch as kernel arguments) zeroes exactly
    the given disjoint ranges -- across launch boundaries and for ranges longer than one 16 K chunk -- and nothing
    else."""
    import numpy as np
    g = torch.Generator().manual_seed(n_ranges)
    lens = torch.randint(1, 40000, (n_ranges,), generator=g).numpy().astype(np.int64)
    gaps = torch.randint(0, 3000, (n_ranges,), generator=g).numpy().astype(np.int64)
    starts = np.cumsum(gaps + np.concatenate([[0], lens[:-1]])).astype(np.int64)
    total = int(starts[-1] + lens[-1] + 100)
    base = torch.randn(total, device=dev)
    ref = base.clone()
    for s, n in zip(starts.tolist(), lens.tolist()):
        ref[s:s + n] = 0
    K.zero_ranges(base, starts, lens)
    torch.cuda.synchronize()
    assert torch.equal(base, ref)


@pytest.mark.parametrize("use_bf16_out", [True, False])
def test_layernorm_twin_matches_cast_path(K, use_bf16_out):
    """LayerNormTwinFn (hip_ops): the fp32 twin equals fp32(bf16 output) exactly, and with both outputs consumed
    (bf16 -> a GEMM-like use, fp32 -> a residual) x / w / b get the gradients of the cast path against fp32 torch."""
    from iit_amd.ops.hip_ops import LayerNormTwinFn, _f32_of
    torch.manual_seed(21)
    T, d = 777, 768
    x = (torch.randn(T, d, device=dev) * 2 + 0.5).requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(d, device=dev))
    b = torch.nn.Parameter(torch.randn(d, device=dev))
    y, y32 = LayerNormTwinFn.apply(x, w, b, 1e-5)
    assert y.dtype == torch.bfloat16 and y32.dtype == torch.float32
    assert torch.equal(y32, y.float())
    g1 = torch.randn(T, d, device=dev)
    g2 = torch.randn(T, d, device=dev)
    loss = (y32 * g2).sum() + ((y.float() * g1).sum() if use_bf16_out else 0.0)
    loss.backward()
    xr = x.detach().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (d,), wr, br, 1e-5)
    ((yr * (g1 + g2 if use_bf16_out else g2)).sum()).backward()
    assert rel_err(x.grad, xr.grad) < 1e-2
    assert rel_err(w.grad, wr.grad) < 1e-2 and rel_err(b.grad, br.grad) < 1e-2
    # the twin attribute is honoured only for the exact tensor (storage and version) it was attached to
    y._iit_f32 = (y.data_ptr(), y._version, y32)
    assert _f32_of(y) is y32
    y.add_(0)  # an in-place change invalidates it (the outputs are not views: in-place ops are allowed)
    assert _f32_of(y) is y

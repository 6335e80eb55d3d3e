"""GPU parity of each HIP kernel (through the C ABI) against the CPU oracle / fp32 references.

Tolerances (protocol P1): GEMM / attention rel-L2 <= 1e-2 vs fp32 accumulation of the same
bf16 operands; norms/elementwise within 1-2 bf16 ulp (rel-L2 <= 8e-3); generators bit-exact.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - these tests need the MI355X box
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import _native as nat  # noqa: E402
from oracle import flite_ref as R  # noqa: E402
from oracle.weights import hash_uniform  # noqa: E402

DEV = "cuda"


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_library_loads_every_symbol():
    lib = nat.load()
    for name in nat.SIGNATURES:
        assert hasattr(lib, name)


@pytest.mark.parametrize("M,N,K", [(1, 64, 64), (256, 256, 64), (300, 200, 128), (1000, 768, 4096),
                                   (8224, 3072, 3072)])
def test_gemm_bias_bf16(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + N)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).bfloat16()
    b = (torch.randn(N, device=DEV, generator=g) * 0.1).bfloat16()
    ref = a.float() @ w.float().t() + b.float()
    out = nat.gemm(a, w, b)
    assert rel(out, ref) < 1e-2
    out32 = nat.gemm(a, w, b, epilogue=nat.EPI_STORE_F32)
    assert rel(out32, ref) < 1e-5


def test_gemm_strided_operands():
    # A with a row stride larger than K (a column slice), W slice
    a_full = torch.randn(500, 320, device=DEV).bfloat16()
    a = a_full[:, :256]
    w = (torch.randn(96, 256, device=DEV) * 0.05).bfloat16()
    out = nat.gemm(a, w, None, epilogue=nat.EPI_STORE_F32)
    assert rel(out, a.float() @ w.float().t()) < 1e-5


def test_gemm_swiglu():
    M, F, K = 777, 1024, 512
    a = torch.randn(M, K, device=DEV).bfloat16()
    wg = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()
    wu = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()
    ref = torch.nn.functional.silu(a.float() @ wg.float().t()) * (a.float() @ wu.float().t())
    out = nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu)
    assert rel(out, ref) < 1e-2


# segments of 300 rows: some waves' rows straddle a segment boundary (per-row gate path), the others take the
# one-round-trip path (rows 0-3 of x through LDS); shared gate rows; no gate at all
@pytest.mark.parametrize("shared", [False, True, None])
def test_gemm_gated_residual(shared):
    M, N, K, T = 1000, 768, 256, 300
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    nseg = (M + T - 1) // T
    gate = torch.randn(nseg, N, device=DEV)
    x0 = torch.randn(M, N, device=DEV)
    y = a.float() @ w.float().t() + b.float()
    ref = x0.clone()
    for s in range(nseg):
        ref[s * T:(s + 1) * T] += y[s * T:(s + 1) * T] * (1.0 if shared is None else gate[0 if shared else s])
    x = x0.clone()
    nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, gate=None if shared is None else gate,
             gate_seg_stride=0 if shared else N, rows_per_seg=T)
    assert rel(x, ref) < 1e-5


# 224-row tiles (gemm.hip use_bm224): on 256 CUs, M = 8224 / 8174 with N = 3072 (also 2F = 3072 for SwiGLU) take
# 2 rounds of 7/8-size tiles instead of 2 full rounds, so the launcher runs MI = 7; 2F = 24576 (the DiT's gate/up:
# 14 rounds of 224 rows against 13 of 256) runs 256-row tiles. Ragged last tiles (8224 = 36 x 224 + 160,
# 8174 = 36 x 224 + 110) and every epilogue those GEMMs use.
@pytest.mark.parametrize("M", [8224, 8174])
def test_gemm_224_row_tiles(M):
    N, K, T = 3072, 128, 4112
    g = torch.Generator(device=DEV).manual_seed(M)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).bfloat16()
    b = (torch.randn(N, device=DEV, generator=g) * 0.1).bfloat16()
    y = a.float() @ w.float().t() + b.float()
    assert rel(nat.gemm(a, w, b), y) < 1e-2
    assert rel(nat.gemm(a, w, b, epilogue=nat.EPI_STORE_F32), y) < 1e-5
    nseg = (M + T - 1) // T
    gate = torch.randn(nseg, N, device=DEV, generator=g)
    x0 = torch.randn(M, N, device=DEV, generator=g)
    ref = x0.clone()
    for s in range(nseg):
        ref[s * T:(s + 1) * T] += y[s * T:(s + 1) * T] * gate[s]
    x = x0.clone()
    nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, gate=gate, gate_seg_stride=N, rows_per_seg=T)
    assert rel(x, ref) < 1e-5
    for F in (1536, 12288):
        wg = (torch.randn(F, K, device=DEV, generator=g) * 0.05).bfloat16()
        wu = (torch.randn(F, K, device=DEV, generator=g) * 0.05).bfloat16()
        sw = nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu)
        assert rel(sw, torch.nn.functional.silu(a.float() @ wg.float().t()) * (a.float() @ wu.float().t())) < 1e-2


# Gated-FF GEMM epilogues store 16-B pieces re-dealt across lanes by v_permlane16_swap (common.h deal8) when the
# output rows are 16-B aligned; a misaligned output view takes the 8-B-store path. Same values: bit-identical.
# Ragged M (8174: a last tile of 110 rows) and F % 32 == 16 (the last 16 output columns of a tile masked).
@pytest.mark.parametrize("M,F", [(8224, 12288), (8174, 3088)])
@pytest.mark.parametrize("epi", ["swiglu", "geglu"])
def test_gemm_gated_wide_stores_bit_identical(M, F, epi):
    K = 512
    g = torch.Generator(device=DEV).manual_seed(M + F)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    wg = (torch.randn(F, K, device=DEV, generator=g) * 0.05).bfloat16()
    wu = (torch.randn(F, K, device=DEV, generator=g) * 0.05).bfloat16()
    e = nat.EPI_SWIGLU_BF16 if epi == "swiglu" else nat.EPI_GEGLU_BF16
    out = nat.gemm(a, wg, epilogue=e, w2=wu)
    gf, uf = a.float() @ wg.float().t(), a.float() @ wu.float().t()
    act = torch.nn.functional.silu(gf) if epi == "swiglu" else torch.nn.functional.gelu(gf, approximate="tanh")
    assert rel(out, act * uf) < 1e-2
    buf = torch.full((M, F + 8), -1.0, device=DEV, dtype=torch.bfloat16)
    view = buf[:, 4:4 + F]  # 8-B aligned rows: the 8-B-store path
    nat.gemm(a, wg, epilogue=e, w2=wu, out=view)
    assert torch.equal(view, out)
    assert bool((buf[:, :4] == -1).all()) and bool((buf[:, 4 + F:] == -1).all())  # nothing stored outside


# Stream-K (flite_gemm_bf16_ws): shapes whose last wave of 256x256 tiles is partial on 256 CUs and whose k-depth
# makes the split pay (gemm.hip choose_sk_tiles), so the launcher cuts that wave's k-iterations evenly over the
# CUs: the 10B down projection, and small grids where one tile is shared by up to ~28 workgroups (fan-in).
@pytest.mark.parametrize("M,N,K", [(8224, 3072, 12288), (2000, 2304, 8192), (1000, 768, 16384), (600, 520, 4096)])
def test_gemm_stream_k(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(K)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).bfloat16()
    b = (torch.randn(N, device=DEV, generator=g) * 0.1).bfloat16()
    ws = nat.gemm_workspace(DEV)
    ref = a.double() @ w.double().t() + b.double()
    # fp32 store: rel-L2 vs fp64 at fp32-accumulation level, same as the data-parallel path
    dp = nat.gemm(a, w, b, epilogue=nat.EPI_STORE_F32)
    sk = nat.gemm(a, w, b, epilogue=nat.EPI_STORE_F32, workspace=ws)
    assert rel(sk, ref) < 1e-5 and rel(dp, ref) < 1e-5
    assert not torch.equal(sk, dp)  # the split path ran (different fp32 summation order)
    # deterministic: the same split and reduction order on every launch (flags reset by the finishers)
    sk2 = nat.gemm(a, w, b, epilogue=nat.EPI_STORE_F32, workspace=ws)
    assert torch.equal(sk, sk2)
    n_cu = ws.numel() // (256 * 256 * 4 + 4)
    assert int(ws[n_cu * 256 * 256 * 4:].view(torch.int32).abs().sum().item()) == 0  # every flag back to 0
    # gated residual (the engine's proj / down GEMMs)
    T = M // 2 if M % 2 == 0 else M
    gate = torch.randn((M + T - 1) // T, N, device=DEV)
    x0 = torch.randn(M, N, device=DEV)
    x = x0.clone()
    nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, gate=gate, gate_seg_stride=N, rows_per_seg=T,
             workspace=ws)
    y = a.float() @ w.float().t() + b.float()
    refx = x0 + y * gate.repeat_interleave(T, dim=0)[:M]
    assert rel(x, refx) < 1e-5
    # bf16 store
    out = nat.gemm(a, w, b, workspace=ws)
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("M,F,K", [(2000, 1152, 8192),    # N = 2F = 2304: 72 tiles, stream-K by the model
                                   (8224, 12288, 3072)])  # the DiT gate/up: 12 rounds + 96 leftover tiles
def test_gemm_stream_k_swiglu(M, F, K):
    a = torch.randn(M, K, device=DEV).bfloat16()
    wg = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()
    wu = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()
    ref = torch.nn.functional.silu(a.float() @ wg.float().t()) * (a.float() @ wu.float().t())
    ws = nat.gemm_workspace(DEV)
    out = nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu, workspace=ws)
    assert rel(out, ref) < 1e-2
    dp = nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu)
    assert rel(dp, ref) < 1e-2
    assert not torch.equal(out, dp)  # the split path ran (different fp32 summation order in the leftover tiles)
    assert torch.equal(out, nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu, workspace=ws))  # deterministic
    n_cu = ws.numel() // (256 * 256 * 4 + 4)
    assert int(ws[n_cu * 256 * 256 * 4:].view(torch.int32).abs().sum().item()) == 0  # every flag back to 0


def _attn_ref(q, k, v, cu_q, cu_k, scale):
    return R.attention_varlen(q.float().cpu(), k.float().cpu(), v.float().cpu(), cu_q.cpu(), cu_k.cpu(), scale)


@pytest.mark.parametrize("bounded", [False, True])
@pytest.mark.parametrize("lens_q,lens_k", [([80, 80], None), ([272, 272], None), ([4112], None),
                                           ([100, 37], [24, 17]), ([130, 5], [512, 0]), ([64], [1])])
def test_attention_varlen(lens_q, lens_k, bounded):
    H, D = 2, 256
    self_attn = lens_k is None
    lens_k = lens_q if self_attn else lens_k
    cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
    g = torch.Generator(device=DEV).manual_seed(sum(lens_q))
    # unit-RMS rows like the QK-normed operands of the model (scores up to ~16)
    q = R.own_rmsnorm(torch.randn(int(cu_q[-1]), H, D, device=DEV, generator=g), None).bfloat16()
    k = R.own_rmsnorm(torch.randn(max(int(cu_k[-1]), 1), H, D, device=DEV, generator=g), None).bfloat16()
    v = torch.randn(max(int(cu_k[-1]), 1), H, D, device=DEV, generator=g).bfloat16()
    out = nat.attn_varlen(q, k, v, cu_q.to(DEV), cu_k.to(DEV), max(lens_q), D ** -0.5,
                          max_score=16.5 if bounded else 0.0)
    ref = _attn_ref(q, k, v, cu_q, cu_k, D ** -0.5)
    assert rel(out, ref) < 1e-2


# Tail split (attention.hip "Schedule"): the partial last q-tile of every (sequence, head) is cut by key ranges
# over the chip and reduced in slab order. Cases: the DiT self (T = 4112: 16-row tails) and cross shapes, ragged
# tails of up to 127 rows, more chunks than key tiles (empty chunks), no keys at all; with max_k, the engine's
# policy (cross-attention: tail chunks first).
@pytest.mark.parametrize("lens_q,lens_k,H", [([4112, 4112], None, 12), ([4112, 4112], [512, 512], 12),
                                             ([300, 200], None, 2), ([130, 255], [24, 17], 2),
                                             ([1000, 77], [700, 0], 3), ([50], [4096], 1)])
def test_attention_tail_split(lens_q, lens_k, H):
    D = 256
    self_attn = lens_k is None
    lens_k = lens_q if self_attn else lens_k
    B = len(lens_q)
    ws = nat.attn_workspace(DEV, B, H)
    assert ws is not None  # every case here is small enough in B*H for the split
    cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
    g = torch.Generator(device=DEV).manual_seed(sum(lens_q) + H)
    q = R.own_rmsnorm(torch.randn(int(cu_q[-1]), H, D, device=DEV, generator=g), None).bfloat16()
    k = R.own_rmsnorm(torch.randn(max(int(cu_k[-1]), 1), H, D, device=DEV, generator=g), None).bfloat16()
    v = torch.randn(max(int(cu_k[-1]), 1), H, D, device=DEV, generator=g).bfloat16()
    args = (q, k, v, cu_q.to(DEV), cu_k.to(DEV), max(lens_q), D ** -0.5)
    split = nat.attn_varlen(*args, max_score=16.5, workspace=ws)
    whole = nat.attn_varlen(*args, max_score=16.5)
    if sum(lens_q) * H * max(lens_k) <= 2 * 4112 * 4112 * 2:
        ref = _attn_ref(q, k, v, cu_q, cu_k, D ** -0.5)
        assert rel(split, ref) < 1e-2
    assert rel(split, whole) < 5e-3  # same math, only the summation order of the tail rows differs
    # deterministic (fixed slab order) and the workspace is left zeroed for the next launch
    again = nat.attn_varlen(*args, max_score=16.5, workspace=ws)
    assert torch.equal(split, again)
    assert int(ws[:4096].view(torch.int32).abs().sum().item()) == 0
    # with the key length known (the engine's call): key ranges of 256-1023 keys dispatch their tail chunks
    # before the full q-tiles (split_first), shorter ones do not split
    policy = nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k))
    assert rel(policy, whole) < 5e-3
    assert torch.equal(policy, nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k)))
    assert int(ws[:4096].view(torch.int32).abs().sum().item()) == 0


def test_attention_spike_rescale():
    # force the online-softmax rescale: one key far above the rest in a late tile (§5.4 rule 26)
    H, D, L = 1, 256, 700
    q = R.own_rmsnorm(torch.randn(L, H, D, device=DEV), None)
    k = R.own_rmsnorm(torch.randn(L, H, D, device=DEV), None)
    k[650] = q[3] * 1.0  # row 3's max jumps at tile 10
    k[90] = -q[3]
    q, k = q.bfloat16(), k.bfloat16()
    v = torch.randn(L, H, D, device=DEV).bfloat16()
    cu = torch.tensor([0, L], dtype=torch.int32)
    out = nat.attn_varlen(q, k, v, cu.to(DEV), cu.to(DEV), L, 1.0)  # scale 1: scores up to 256
    ref = _attn_ref(q, k, v, cu, cu, 1.0)
    assert rel(out, ref) < 1e-2


# 3072: the one-workgroup-per-row kernel of the DiT width (bf16 rows: the round-6 residual stream);
# 602 rows: a partial last group of the 4-row kernel; 603 rows of 251: a lone last row and row pairs that straddle a
# modulation segment
@pytest.mark.parametrize("rows,T", [(602, 250), (603, 251)])
@pytest.mark.parametrize("D", [512, 3072])
@pytest.mark.parametrize("in_bf16", [False, True])
def test_rmsnorm_modulate(in_bf16, D, rows, T):
    x = torch.randn(rows, D, device=DEV) * 3
    if in_bf16:
        x = x.bfloat16()
    w = (1 + 0.1 * torch.randn(D, device=DEV)).bfloat16()
    nseg = (rows + T - 1) // T
    shift = torch.randn(nseg, D, device=DEV) * 0.1
    scale = torch.randn(nseg, D, device=DEV) * 0.1
    out = nat.rmsnorm_modulate(x, w, shift, scale, seg_rows=T)
    xf = x.float().cpu()
    n = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float().cpu()
    seg = torch.arange(rows) // T
    ref = n * (1 + scale.cpu()[seg]) + shift.cpu()[seg]
    assert rel(out, ref) < 4e-3


def test_rope_tables_match_reference(golden):
    cos, sin = nat.rope_tables(12, 20, 16, 10000.0, round_bf16=False)
    # fp32 tables: device cosf/sinf vs torch CPU within 2 ulp-ish
    assert (cos.cpu() - golden["op.rope.cos"]).abs().max() < 2e-6
    assert (sin.cpu() - golden["op.rope.sin"]).abs().max() < 2e-6
    cb, sb = nat.rope_tables(12, 20, 16, 10000.0, round_bf16=True)
    mism = (cb.cpu() != golden["op.rope_bf16.cos"]).float().mean().item()
    assert mism < 1e-3  # bf16 rounding of 1-ulp-different fp32 values can flip a handful of entries


@pytest.mark.parametrize("H", [2, 3, 12])  # heads run in pairs: odd counts leave a half-empty pair
def test_rope_qknorm(H):
    rows, T = 300, 150
    x = torch.randn(rows, 3 * H * 256, device=DEV).bfloat16()
    cos, sin = nat.rope_tables(12, 13, 16, 10000.0, round_bf16=True)
    assert cos.shape[0] >= T
    cos, sin = cos[:T].contiguous(), sin[:T].contiguous()
    y = x.clone()
    nat.rope_qknorm_(y, heads=2 * H, rope_heads=2 * H, cos=cos, sin=sin, tokens_per_seq=T)
    xc = x.float().cpu().reshape(rows, 3, H, 256)
    tok = torch.arange(rows) % T
    c, s = cos.cpu()[tok][:, None, :], sin.cpu()[tok][:, None, :]
    for part in range(2):
        ref = R.own_rmsnorm(R.apply_rotary_emb(xc[:, part], c, s), None)
        got = y.float().cpu().reshape(rows, 3, H, 256)[:, part]
        assert rel(got, ref) < 4e-3
    assert torch.equal(y[:, 2 * H * 256:], x[:, 2 * H * 256:])  # v untouched
    # norm only (cross-attention q), odd head count, rotation on a prefix of the heads
    z = x.clone()
    nat.rope_qknorm_(z, heads=H, rope_heads=0)
    refq = R.own_rmsnorm(xc[:, 0], None)
    assert rel(z.float().cpu().reshape(rows, 3, H, 256)[:, 0], refq) < 4e-3
    assert torch.equal(z[:, H * 256:], x[:, H * 256:])
    if H >= 2:
        u = x.clone()
        nat.rope_qknorm_(u, heads=H, rope_heads=1, cos=cos, sin=sin, tokens_per_seq=T)
        got = u.float().cpu().reshape(rows, 3, H, 256)[:, 0]
        assert rel(got[:, :1], R.own_rmsnorm(R.apply_rotary_emb(xc[:, 0, :1], c, s), None)) < 4e-3
        assert rel(got[:, 1:], R.own_rmsnorm(xc[:, 0, 1:], None)) < 4e-3


def test_timestep_embedding_quantized(golden):
    t = golden["op.temb_bf16t.t"].to(DEV)
    emb = nat.timestep_embedding(t, 512, quantize=True)
    ref = golden["op.temb_bf16t.out"].bfloat16().float()
    assert (emb.float().cpu() - ref).abs().max() < 8e-3  # 1 bf16 ulp at |x| <= 1


def test_init_param_bit_exact():
    for name, n, std in [("blocks.0.self_attn.qkv.weight", 100003, 0.02), ("register_tokens", 8192, 0.02),
                         ("x", 5000, 1.0)]:
        t = torch.empty(n, device=DEV, dtype=torch.float32)
        nat.init_param_(t, name, seed=3, std=std)
        ref = torch.from_numpy(hash_uniform(name, n, std, seed=3))
        assert torch.equal(t.cpu(), ref)
        tb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
        nat.init_param_(tb, name, seed=3, std=std)
        assert torch.equal(tb.cpu(), ref.bfloat16())


# The 256-query-row kernel (attention_q256.hip): bounded launches over >= 1024 keys with a workspace sized by
# attn_workspace(..., max_q, max_k) and max_k given. Its plan runs some full q-tiles whole, others as two key halves,
# and the tail rows as key chunks. Against the fp32 reference and the 128-row kernel (same launch without max_k).
# Cases: the DiT self-attention (T = 4112, 16-row tails), the 1344x896 length (T = 4720, 112-row tails), one sequence
# (every full tile split), unequal lengths (a short sequence's q-tiles and tails end early), a length that is a
# multiple of 256 (no tail), a key range not a multiple of 32, cross-shaped keys.
@pytest.mark.parametrize("lens_q,lens_k,H", [([4112, 4112], None, 12), ([4720], None, 4), ([1300], None, 1),
                                             ([3000, 1500], None, 3), ([2048], None, 2), ([700, 900], [1100, 1037], 2),
                                             ([4112], [1536], 12)])
def test_attention_q256(lens_q, lens_k, H):
    D = 256
    lens_k = lens_q if lens_k is None else lens_k
    B = len(lens_q)
    ws = nat.attn_workspace(DEV, B, H, max(lens_q), max(lens_k))
    old_ws = nat.attn_workspace(DEV, B, H)
    assert ws is not None and (old_ws is None or ws.numel() >= old_ws.numel())
    cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
    g = torch.Generator(device=DEV).manual_seed(sum(lens_q) + 7 * H)
    q = R.own_rmsnorm(torch.randn(int(cu_q[-1]), H, D, device=DEV, generator=g), None).bfloat16()
    k = R.own_rmsnorm(torch.randn(int(cu_k[-1]), H, D, device=DEV, generator=g), None).bfloat16()
    v = torch.randn(int(cu_k[-1]), H, D, device=DEV, generator=g).bfloat16()
    args = (q, k, v, cu_q.to(DEV), cu_k.to(DEV), max(lens_q), D ** -0.5)
    nat.attn_set_q256(True)
    try:
        new = nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k))
        again = nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k))
    finally:
        nat.attn_set_q256(2)
    assert int(ws[:4096].view(torch.int32).abs().sum().item()) == 0  # counters left zeroed
    nat.attn_set_q256(0)
    try:
        old = nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k))  # the 128-row kernel
    finally:
        nat.attn_set_q256(2)
    # the two kernels share one workspace (the engine's): the 128-row kernel's slabs must not disturb the 256-row
    # kernel's counters
    nat.attn_set_q256(True)
    try:
        after = nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max(lens_k))
    finally:
        nat.attn_set_q256(2)
    assert torch.equal(new, after)
    assert torch.isfinite(new.float()).all()
    ref = torch.empty(q.shape, dtype=torch.float32, device=DEV)  # fp32 reference per (sequence, head), on the GPU
    for b in range(B):
        qs, ks = slice(int(cu_q[b]), int(cu_q[b + 1])), slice(int(cu_k[b]), int(cu_k[b + 1]))
        for h in range(H):
            ref[qs, h] = torch.softmax(q[qs, h].float() @ k[ks, h].float().T * D ** -0.5, -1) @ v[ks, h].float()
    assert rel(new, ref) < 1e-2
    print(f"q256 {lens_q} x {lens_k} H={H}: rel vs fp32 {rel(new, ref):.2e} (128-row kernel {rel(old, ref):.2e})")
    assert rel(new, old) < 5e-3  # same math; split halves and chunk sums change the summation order only
    assert torch.equal(new, again)  # deterministic whichever split piece arrives last

"""Training-mode HIP ops vs torch autograd of the CPU oracle math (fp32, same inputs).

Tolerance: relative L2 <= 1e-5 on every gradient (north-star fp32 tolerance), 1e-6 where the op is a
single GEMM; integer arg-max outputs bit-exact."""
import pytest
import torch
import torch.nn.functional as F

from oracle import ptv3_ref
from splatformer_amd import ptv3_ops as ops
from splatformer_amd import train_ops as tops

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K,dact", [(1000, 64, 96, 0), (777, 384, 96, 1), (300, 128, 512, 2), (64, 23, 128, 3)])
def test_linear_bwd_data(device, M, N, K, dact):
    g = torch.Generator().manual_seed(M)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    dy = torch.randn(M, N, generator=g)
    pre = torch.randn(M, K, generator=g)
    if dact == 3:
        pre = torch.tanh(pre)
    rs = (torch.rand(M, generator=g) > 0.3).float() / 0.7
    base = torch.randn(M, K, generator=g)
    ref = (dy @ w) * rs[:, None]
    if dact == 1:
        x = pre.clone().requires_grad_()
        F.gelu(x).backward(torch.ones_like(x))
        ref = ref * x.grad
    elif dact == 2:
        ref = ref * (pre > 0).float()
    elif dact == 3:
        ref = ref * (1 - pre * pre)
    wt = tops.transpose(w.to(device))
    assert torch.equal(wt.cpu(), w.T.contiguous())
    out = base.to(device).clone()
    tops.linear_bwd_data(dy.to(device), wt, rowscale=rs.to(device), dact=dact, dact_pre=pre.to(device), out=out,
                         accumulate=True)
    assert rel_l2(out, ref + base) < 2e-6


@pytest.mark.parametrize("M,N,K", [(100000, 192, 64), (777, 384, 128), (33, 1536, 512), (37759, 768, 256),
                                   (5003, 100, 36), (40, 288, 96)])
def test_linear_wgrad(device, M, N, K):
    g = torch.Generator().manual_seed(N)
    dy = torch.randn(M, N, generator=g)
    x = torch.randn(M, K, generator=g)
    dw0 = torch.randn(N, K, generator=g)
    db0 = torch.randn(N, generator=g)
    dw, db = dw0.to(device), db0.to(device)
    tops.linear_wgrad(dy.to(device), x.to(device), dw, db)
    assert rel_l2(dw, dw0 + dy.double().T @ x.double()) < 1e-5
    assert rel_l2(db, db0 + dy.double().sum(0)) < 1e-5


@pytest.mark.parametrize("M,N,K", [(37759, 768, 256), (5003, 128, 64)])
def test_linear_wgrad_reference_precision(device, M, N, K):
    """Weight gradient under ops.precision("amp") (three bf16 term products, 16-bit significands): finer than the
    reference autocast's fp16-operand product, coarser than the fp32-accurate default."""
    g = torch.Generator().manual_seed(K)
    dy = torch.randn(M, N, generator=g)
    x = torch.randn(M, K, generator=g)
    exact = dy.double().T @ x.double()
    e16 = rel_l2(dy.half().double().T @ x.half().double(), exact)
    dw = torch.zeros(N, K, device=device)
    with ops.precision("amp"):
        tops.linear_wgrad(dy.to(device), x.to(device), dw, None)
    e_amp = rel_l2(dw, exact)
    dw.zero_()
    tops.linear_wgrad(dy.to(device), x.to(device), dw, None)
    e_32 = rel_l2(dw, exact)
    assert e_32 < e_amp <= e16, (e_32, e_amp, e16)


@pytest.mark.parametrize("n,cin,cout,dup", [(3000, 64, 64, False), (2000, 96, 128, True), (500, 256, 256, False)])
def test_subm_conv_bwd_data(device, n, cin, cout, dup):
    g = torch.Generator().manual_seed(n)
    grid = torch.randint(0, 24, (n, 3), generator=g).int()
    if dup:
        grid[n // 2:n // 2 + 50] = grid[:50]  # duplicate voxels -> centre maps to the lowest index
    batch = torch.zeros(n, dtype=torch.int32)
    nbr = ptv3_ref.subm_neighbors(grid, batch)
    w = torch.randn(cout, 3, 3, 3, cin, generator=g) / (27 * cin) ** 0.5
    b = torch.randn(cout, generator=g)
    x = torch.randn(n, cin, generator=g, requires_grad=True)
    dy = torch.randn(n, cout, generator=g)
    ptv3_ref.subm_conv(x, nbr, w, b).backward(dy)
    smap = ops.subm_neighbors(grid.to(device), None)
    wt = tops.transpose(w.reshape(cout, 27 * cin).to(device))
    base = torch.randn(n, cin, generator=g)
    dx = base.to(device).clone()
    tops.subm_conv_bwd_data(dy.to(device), smap, wt, dx)
    assert rel_l2(dx, x.grad + base) < 1e-5


@pytest.mark.parametrize("n,heads,C,mag,gmag", [(1000, 2, 64, 1.0, 1.0), (777, 4, 96, 1.0, 1.0), (300, 8, 128, 1.0, 1.0),
                                               (100, 2, 32, 1.0, 1.0), (1500, 16, 256, 1.0, 1.0),
                                               (1000, 4, 64, 2.5, 1e4), (640, 4, 96, 1e-3, 1e-5),
                                               (129, 4, 128, 1.0, 1.0)])
def test_window_attention_bwd(device, n, heads, C, mag, gmag):
    """Default (fp16x2 two-pass) backward vs fp32 autograd of the reference math: ragged last windows (keys in two
    windows), a single short window (n < 128), peaked softmax (|qkv| x 2.5: logits std 6, large dO) and tiny operands (the
    per-item power-of-two scales)."""
    g = torch.Generator().manual_seed(n + C)
    qkv = (torch.randn(n, 3 * C, generator=g) * mag).requires_grad_()
    order = torch.randperm(n, generator=g)
    inverse = torch.empty_like(order)
    inverse[order] = torch.arange(n)
    K = min(n, 128)
    pad, unpad = ptv3_ref.get_padding_and_inverse(torch.tensor([n]), K)
    q, k, v = qkv[order[pad]].reshape(-1, K, 3, heads, C // heads).permute(2, 0, 3, 1, 4).unbind(0)
    att = torch.softmax((q * (C // heads) ** -0.5) @ k.transpose(-2, -1), -1)
    ref = (att @ v).transpose(1, 2).reshape(-1, C)[unpad[inverse]]
    dout = torch.randn(n, C, generator=g) * gmag
    ref.backward(dout)
    tab = ops.window_table([n], K)
    win = torch.tensor(tab, dtype=torch.int32).to(device)
    dqkv = tops.window_attention_bwd(qkv.detach().to(device), order.int().to(device), win, len(tab), K, heads, C,
                                     dout.to(device))
    assert rel_l2(dqkv, qkv.grad) < 1e-5
    if mag == 1.0 and gmag == 1.0:  # reference-precision mode: single fp16 products (fp16-operand error)
        with ops.precision("amp"):
            dqa = tops.window_attention_bwd(qkv.detach().to(device), order.int().to(device), win, len(tab), K, heads,
                                            C, dout.to(device))
        assert 2e-5 < rel_l2(dqa, qkv.grad) < 5e-3, rel_l2(dqa, qkv.grad)


@pytest.mark.parametrize("K", [1024, 256])
@pytest.mark.parametrize("heads,C", [(2, 32), (4, 96), (8, 256)])
def test_window_attention_varlen_bwd(device, K, heads, C):
    """enable_flash=True backward vs fp64 autograd of the oracle's cu_seqlens restatement: batches of n < K,
    n == K, ragged n > K (keys shared by two windows) and 2K."""
    counts = [700, K, 2 * K + 333, 2 * K, 5]
    n = sum(counts)
    offset = torch.tensor(counts).cumsum(0)
    g = torch.Generator().manual_seed(K + C + 1)
    qkv = torch.randn(n, 3 * C, generator=g, dtype=torch.float64)
    order = torch.cat([torch.randperm(c, generator=g) + (int(offset[i]) - c) for i, c in enumerate(counts)])
    inverse = torch.empty_like(order)
    inverse[order] = torch.arange(n)
    point = ptv3_ref.Point(offset=offset, serialized_order=order[None], serialized_inverse=inverse[None])
    qkv_ref = qkv.clone().requires_grad_()
    out = ptv3_ref.serialized_attention_flash(qkv_ref, point, C, heads, K, 0)
    dout = torch.randn(n, C, generator=g, dtype=torch.float64)
    out.backward(dout)
    tab = ops.window_table_varlen_np(offset.tolist(), K)
    win3 = torch.from_numpy(tab).to(device)
    dqkv = tops.window_attention_varlen_bwd(qkv.float().to(device), order.int().to(device), win3, tab.shape[0], K,
                                            heads, C, dout.float().to(device))
    assert rel_l2(dqkv, qkv_ref.grad) < 1e-5


def test_layernorm_bwd_ops(device):
    g = torch.Generator().manual_seed(3)
    for C in (64, 96, 128, 256, 512, 48):
        M = 999
        x = (torch.randn(M, C, generator=g) * 2 + 0.5).requires_grad_()
        ga, be = torch.randn(C, generator=g), torch.randn(C, generator=g)
        dy = torch.randn(M, C, generator=g)
        dr = torch.randn(M, C, generator=g)
        F.layer_norm(x, (C,), ga, be, 1e-5).backward(dy)
        got = tops.layernorm_bwd(x.detach().to(device), ga.to(device), dy.to(device), 1e-5, dres=dr.to(device))
        assert rel_l2(got, x.grad + dr) < 1e-5
        # fused block tail: x1 = x + LN_c(u); h = LN1(x1)
        u = torch.randn(M, C, generator=g, requires_grad=True)
        xx = torch.randn(M, C, generator=g)
        gc, bc = torch.randn(C, generator=g), torch.randn(C, generator=g)
        g1, b1 = torch.randn(C, generator=g), torch.randn(C, generator=g)
        x1 = (xx + F.layer_norm(u, (C,), gc, bc, 1e-5)).detach().requires_grad_()
        h = F.layer_norm(x1, (C,), g1, b1, 1e-5)
        dh = torch.randn(M, C, generator=g)
        dx2 = torch.randn(M, C, generator=g)
        h.backward(dh)
        dx1_ref = x1.grad + dx2
        F.layer_norm(u, (C,), gc, bc, 1e-5).backward(dx1_ref)
        dx1, du = tops.cpe_ln_bwd(u.detach().to(device), x1.detach().to(device), gc.to(device), g1.to(device),
                                  dx2.to(device), dh.to(device), 1e-5)
        assert rel_l2(dx1, dx1_ref) < 1e-5
        assert rel_l2(du, u.grad) < 1e-5


@pytest.mark.parametrize("M,C", [(5000, 64), (777, 256), (3, 96)])
def test_bn_train_fwd_bwd(device, M, C):
    g = torch.Generator().manual_seed(M)
    bn = torch.nn.BatchNorm1d(C, eps=1e-3, momentum=0.01)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g))
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    bn_dev = torch.nn.BatchNorm1d(C, eps=1e-3, momentum=0.01).to(device)
    bn_dev.load_state_dict(bn.state_dict())
    x = (torch.randn(M, C, generator=g) * 3 + 1).requires_grad_()
    res = torch.randn(M // 2 + 1, C, generator=g)
    ridx = torch.randint(0, M // 2 + 1, (M,), generator=g).int()
    bn.train()
    y_ref = F.gelu(bn(x)) + res[ridx.long()]
    dy = torch.randn(M, C, generator=g)
    y_ref.backward(dy)
    y, st = tops.bn_train_forward(x.detach().to(device), bn_dev, 1, residual=res.to(device),
                                  residual_idx=ridx.to(device))
    assert rel_l2(y, y_ref) < 1e-5
    assert rel_l2(bn_dev.running_mean, bn.running_mean) < 1e-6
    assert rel_l2(bn_dev.running_var, bn.running_var) < 1e-6
    dx = tops.bn_act_bwd(st, bn_dev, 1, dy.to(device))
    assert rel_l2(dx, x.grad) < 1e-5


def test_segment_ops(device):
    g = torch.Generator().manual_seed(5)
    n, C = 4000, 96
    cluster = torch.randint(0, 900, (n,), generator=g)
    _, cluster = torch.unique(cluster, return_inverse=True)
    m = int(cluster.max()) + 1
    sidx = torch.sort(cluster, stable=True).indices
    counts = torch.bincount(cluster, minlength=m)
    idx_ptr = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(counts, 0)])
    x = torch.randn(n, C, generator=g, requires_grad=True)
    seg = cluster
    y_ref = torch.full((m, C), -float("inf")).scatter_reduce(0, seg[:, None].expand(n, C), x, reduce="amax",
                                                            include_self=True)
    dy = torch.randn(m, C, generator=g)
    y_ref.backward(dy)
    y, arg = tops.segment_max_arg(x.detach().to(device), idx_ptr.int().to(device), sidx.int().to(device), m)
    assert torch.equal(y.cpu(), y_ref.detach())
    dx = tops.segment_max_bwd(dy.to(device), arg, n)
    assert rel_l2(dx, x.grad) < 1e-6
    s = tops.segment_sum(x.detach().to(device), idx_ptr.int().to(device), sidx.int().to(device), m)
    s_ref = torch.zeros(m, C).index_add_(0, seg, x.detach())
    assert rel_l2(s, s_ref) < 1e-6


def test_act_bwd_and_adam(device):
    g = torch.Generator().manual_seed(6)
    dy = torch.randn(500, 23, generator=g)
    o = torch.tanh(torch.randn(500, 23, generator=g))
    got = tops.act_bwd(dy.to(device), o.to(device), 3, ncols=3)
    ref = dy.clone()
    ref[:, :3] *= 1 - o[:, :3] ** 2
    assert rel_l2(got, ref) < 1e-6
    # clip_grad_norm_(2.0) + Adam(eps 1e-15) for 3 steps vs torch.optim
    ps = [torch.randn(300, 64, generator=g), torch.randn(192, generator=g)]
    ref_p = [p.clone().requires_grad_() for p in ps]
    opt = torch.optim.Adam(ref_p, lr=3e-5, eps=1e-15)
    dev_p = [p.to(device) for p in ps]
    m1 = [torch.zeros_like(p) for p in dev_p]
    m2 = [torch.zeros_like(p) for p in dev_p]
    for step in range(1, 4):
        grads = [torch.randn(p.shape, generator=g) * 3 for p in ps]
        for p, gr in zip(ref_p, grads):
            p.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ref_p, 2.0)
        opt.step()
        dg = [gr.to(device) for gr in grads]
        coef, _ = tops.grad_clip_coef(dg, 2.0)
        for p, gr, a, b in zip(dev_p, dg, m1, m2):
            tops.adam_step(p, gr, a, b, step, 3e-5, eps=1e-15, grad_scale=coef)
    for p, r in zip(dev_p, ref_p):
        assert rel_l2(p, r) < 1e-6


def test_drop_mask(device):
    """sfx_drop_mask: values in {0, 1/keep}, keep fraction within 5 sigma, deterministic per seed."""
    n, keep = 200_000, 0.7
    a = tops.drop_mask(n, keep, 12345, device)
    b = tops.drop_mask(n, keep, 12345, device)
    c = tops.drop_mask(n, keep, 12346, device)
    assert torch.equal(a, b) and not torch.equal(a, c)
    vals = set(torch.unique(a).tolist())
    assert vals <= {0.0, float(torch.tensor(1.0) / torch.tensor(keep))}
    frac = float((a > 0).float().mean())
    sigma = (keep * (1 - keep) / n) ** 0.5
    assert abs(frac - keep) < 5 * sigma, frac
    # neighbouring elements are not correlated (the hash decorrelates consecutive counters)
    k = (a > 0).float()
    both = float((k[1:] * k[:-1]).mean())
    assert abs(both - keep * keep) < 0.01


@pytest.mark.parametrize("C,M", [(64, 3001), (96, 2050), (128, 1999), (256, 1037),
                                 # last round at most half full: split tails (csrc/mlp.hip run_split)
                                 (128, 512 * 64 + 2000), (256, 256 * 64 + 1000)])
def test_block_mlp_train_fwd_bwd(device, C, M):
    """Fused training MLP tail (csrc/mlp.hip MLP_TRAIN / MLP_BWD) vs fp64 autograd of LN2 -> fc1 -> GELU -> fc2 ->
    DropPath row scale -> + shortcut: y, the stored pre-activation z, and the LN2-output gradient dh2."""
    g = torch.Generator().manual_seed(C + M)
    ln2 = torch.nn.LayerNorm(C)
    fc1, fc2 = torch.nn.Linear(C, 4 * C), torch.nn.Linear(4 * C, C)
    with torch.no_grad():
        ln2.weight.copy_(torch.rand(C, generator=g) + 0.5)
        ln2.bias.copy_(torch.randn(C, generator=g) * 0.1)
        for lin in (fc1, fc2):
            lin.weight.copy_(torch.randn(lin.weight.shape, generator=g) / lin.weight.shape[1] ** 0.5)
            lin.bias.copy_(torch.randn(lin.bias.shape, generator=g) * 0.1)
    x2 = torch.randn(M, C, generator=g) * 2 + 0.3
    x2[7] *= 1e3  # rows far apart in magnitude (per-row scales)
    rs = (torch.rand(M, generator=g) > 0.3).float() / 0.7
    dy = torch.randn(M, C, generator=g)
    # fp64 reference
    xd = x2.double()
    h2 = F.layer_norm(xd, (C,), ln2.weight.double(), ln2.bias.double(), ln2.eps).detach().requires_grad_()
    z_ref = h2 @ fc1.weight.double().T + fc1.bias.double()
    y_ref = xd + rs.double()[:, None] * (F.gelu(z_ref) @ fc2.weight.double().T + fc2.bias.double())
    y_ref.backward(dy.double())
    y1_ref = (xd + (F.gelu(z_ref) @ fc2.weight.double().T + fc2.bias.double())).detach()
    dev_mods = [m.to(device) for m in (ln2, fc1, fc2)]
    z = torch.empty(M, 4 * C, device=device)
    y = ops.block_mlp_train(x2.to(device), *dev_mods, z, rowscale=rs.to(device))
    # y vs fp64 on the whole output (fp32 rounding of x2 + branch included), and the branch alone on the rows of
    # ordinary magnitude (row 7's 1e3-scale x2 leaves 6e-5 of output rounding in y - x2)
    keep = torch.arange(M) != 7
    assert rel_l2(z, z_ref) < 2e-6
    assert rel_l2(y, y_ref) < 1e-6
    assert rel_l2((y - x2.to(device))[keep.to(device)], (y_ref - xd)[keep]) < 2e-6
    dh2 = ops.block_mlp_bwd(dy.to(device), *dev_mods, z, rowscale=rs.to(device))
    assert rel_l2(dh2, h2.grad) < 2e-6
    # no mask: rowscale None
    y1 = ops.block_mlp_train(x2.to(device), *dev_mods, z)
    assert rel_l2(y1, y1_ref) < 1e-6
    assert rel_l2((y1 - x2.to(device))[keep.to(device)], (y1_ref - xd)[keep]) < 2e-6
    # reference-precision mode (ops.precision("amp")): one fp16 product per block -- fp16-operand error (~1e-3
    # relative), far above the default's and bounded by it
    with ops.precision("amp"):
        za = torch.empty(M, 4 * C, device=device)
        ya = ops.block_mlp_train(x2.to(device), *dev_mods, za, rowscale=rs.to(device))
        dha = ops.block_mlp_bwd(dy.to(device), *dev_mods, za, rowscale=rs.to(device))
    e_z, e_y = rel_l2(za, z_ref), rel_l2((ya - x2.to(device))[keep.to(device)], (y_ref - xd)[keep])
    e_d = rel_l2(dha, h2.grad)
    assert all(2e-5 < e < 5e-3 for e in (e_z, e_y, e_d)), (e_z, e_y, e_d)

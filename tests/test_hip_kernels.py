"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (MI355X only).

Inputs are rounded to bf16 first, so the reference sees exactly the kernel's operands; the
remaining differences are fp32 accumulation order and the bf16 rounding of outputs.
Asymmetric data everywhere (guide: symmetric operands hide transposes).
"""
import math

import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.ops import reference as R

pytestmark = pytest.mark.gpu

dev = "cuda"


def H():
    from distributed_tensorflow_for_dcgan_amd.ops import hip
    return hip


def bf(t):
    return t.to(torch.bfloat16).contiguous()


def close(out, ref, rel=1.5e-2, name=""):
    out = out.float()
    ref = ref.float()
    scale = ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= rel * scale, "%s: max err %.3e vs scale %.3e" % (name, err, scale)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1).mul(scale).to(dev)


@pytest.mark.parametrize("B,Hs,Ci,Co", [(4, 16, 64, 128), (2, 8, 128, 256), (3, 7, 64, 64), (2, 32, 64, 128)])
def test_conv2d_same_fwd(B, Hs, Ci, Co):
    h = H()
    x = bf(rnd(B, Hs, Hs, Ci, seed=1))
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=2)
    wp = h.pack_conv_weight(w, "conv", "fwd")
    bias = rnd(Co, scale=0.1, seed=3)
    y = h.conv2d_same(x, wp, Co, bias=bias, out_f32=True)
    ref = R.conv2d_same(x.float(), wp.float().reshape(25, Co, Ci).transpose(1, 2).reshape(5, 5, Ci, Co), bias)
    close(y, ref, 2e-3, "conv fwd")


def test_conv2d_same_act_stats_bf16_all_tiles():
    h = H()
    B, Hs, Ci, Co = 4, 16, 64, 128
    x = bf(rnd(B, Hs, Hs, Ci, seed=4))
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=5)
    wp = h.pack_conv_weight(w, "conv", "fwd")
    wref = wp.float().reshape(25, Co, Ci).transpose(1, 2).reshape(5, 5, Ci, Co)
    ref_pre = R.conv2d_same(x.float(), wref)
    for cfg in list(h.IGEMM_CFGS) + [c + 100 for c in h.IGEMM_CFGS]:  # both staging variants
        if h.IGEMM_CFGS[cfg % 100][1] == 16:
            continue
        y, st = h.conv2d_same(x, wp, Co, act="lrelu", stats=True, cfg=cfg)
        close(y, R.lrelu(ref_pre), 1.5e-2, "conv lrelu cfg%d" % cfg)
        s = st.sum(0)
        close(s[0], ref_pre.reshape(-1, Co).sum(0), 2e-3, "stats sum cfg%d" % cfg)
        close(s[1], ref_pre.reshape(-1, Co).pow(2).sum(0), 2e-3, "stats sumsq cfg%d" % cfg)


@pytest.mark.parametrize("B,Hi,Ho,Ci,Co", [(4, 4, 8, 128, 64), (2, 8, 16, 64, 128), (2, 4, 7, 64, 64),
                                          (2, 16, 32, 128, 64), (2, 32, 64, 64, 3)])
def test_conv2d_transpose_same(B, Hi, Ho, Ci, Co):
    h = H()
    x = bf(rnd(B, Hi, Hi, Ci, seed=6))
    w = rnd(5, 5, Co, Ci, scale=0.05, seed=7)
    wp = h.pack_conv_weight(w, "deconv", "fwd")
    bias = rnd(Co, scale=0.1, seed=8)
    y, st = h.conv2d_transpose_same(x, wp, Co, (Ho, Ho), bias=bias, out_f32=True, stats=True)
    ref = R.conv2d_transpose_same(x.float(), wp.float().reshape(5, 5, Co, Ci), (Ho, Ho), bias)
    close(y, ref, 2e-3, "deconv")
    close(st.sum(0)[0], ref.reshape(-1, Co).sum(0), 3e-3, "deconv stats")


def test_dgrad_is_adjoint():
    """D dgrad = deconv with the natural HWIO weight; G dgrad = conv with the transposed one."""
    h = H()
    B, Hs, Ci, Co = 2, 16, 64, 128
    x = rnd(B, Hs, Hs, Ci, seed=9).requires_grad_(True)
    w = bf(rnd(5, 5, Ci, Co, scale=0.05, seed=10)).float()
    dy = bf(rnd(B, 8, 8, Co, seed=11))
    y = R.conv2d_same(x, w)
    (gx,) = torch.autograd.grad(y, x, dy.float())
    out = h.conv2d_transpose_same(dy, h.pack_conv_weight(w, "conv", "dgrad"), Ci, (Hs, Hs), out_f32=True)
    close(out, gx, 2e-3, "conv dgrad")
    # G deconv dgrad
    xd = rnd(B, 8, 8, Co, seed=12).requires_grad_(True)
    wd = bf(rnd(5, 5, Ci, Co, scale=0.05, seed=13)).float()  # [5,5,out=Ci,in=Co]
    yd = R.conv2d_transpose_same(xd, wd, (Hs, Hs))
    dyd = bf(rnd(B, Hs, Hs, Ci, seed=14))
    (gxd,) = torch.autograd.grad(yd, xd, dyd.float())
    outd = h.conv2d_same(dyd, h.pack_conv_weight(wd, "deconv", "dgrad"), Co, out_f32=True)
    close(outd, gxd, 2e-3, "deconv dgrad")


def test_im2col_and_plain_gemm_3ch():
    h = H()
    B, Hs, C, Co = 4, 64, 3, 64
    x = bf(rnd(B, Hs, Hs, C, seed=15))
    col = h.im2col_s2(x, 80)
    w = bf(rnd(5, 5, C, Co, scale=0.05, seed=16)).float()
    bt = h.pack_im2col_weight(w, "conv", 80)
    y = h.gemm_plain(col, bt, out_f32=True)
    ref = R.conv2d_same(x.float(), w).reshape(-1, Co)
    close(y, ref, 2e-3, "im2col conv")


@pytest.mark.parametrize("B,Hs,C,kpad", [(3, 64, 3, 80), (2, 28, 1, 32), (2, 14, 4, 112), (5, 7, 3, 96)])
def test_im2col_exact(B, Hs, C, kpad):
    """im2col_s2 is a pure copy: bit-exact against an unfold of the TF-SAME padded input
    (compile-time C = 3 / 1 paths and the generic one, odd sizes, extra K padding)."""
    import torch.nn.functional as F
    h = H()
    x = bf(rnd(B, Hs, Hs, C, seed=17))
    col = h.im2col_s2(x, kpad)
    Ho = -(-Hs // 2)
    tot = max((Ho - 1) * 2 + 5 - Hs, 0)
    pl = tot // 2
    xp = F.pad(x.permute(0, 3, 1, 2).float(), (pl, tot - pl, pl, tot - pl))
    u = F.unfold(xp, 5, stride=2)  # [B, C*25, Ho*Wo], k = c*25 + tap
    ref = u.reshape(B, C, 25, Ho * Ho).permute(0, 3, 2, 1).reshape(B * Ho * Ho, 25 * C)
    assert torch.equal(col[:, :25 * C].float(), ref)
    assert not col[:, 25 * C:].float().any()


IG3 = [200, 201, 202, 203, 204, 205, 210, 211, 212, 213, 214, 215, 206, 207, 216, 217, 218]  # 2x6..2x8: 8 waves


@pytest.mark.parametrize("bkn", [0, 1])
def test_igemm3_conv_all_tiles_layouts_splits(bkn):
    """v3 kernel: every tile / stage count, both weight layouts, split-K 1/3/4 (in-kernel
    reduction), fused lrelu + BN stats; split-K results are bitwise reproducible."""
    h = H()
    B, Hs, Ci, Co = 4, 16, 128, 256
    x = bf(rnd(B, Hs, Hs, Ci, seed=40))
    w = bf(rnd(5, 5, Ci, Co, scale=0.05, seed=41))          # HWIO = [25][Ci][Co] = bkn layout
    wt = h.pack_conv_weight(w.float(), "conv", "fwd")        # [25][Co][Ci]
    ref_pre = R.conv2d_same(x.float(), w.float())
    wp = w.reshape(25, Ci, Co).contiguous() if bkn else wt
    for cfg in IG3:
        for splits in (1, 3, 4):
            y, st = h.conv2d_same(x, wp, Co, act="lrelu", stats=True, cfg=cfg, bkn=bool(bkn), splits=splits)
            tag = "cfg%d bkn%d s%d" % (cfg, bkn, splits)
            close(y, R.lrelu(ref_pre), 1.5e-2, tag)
            s = st.sum(0)
            close(s[0], ref_pre.reshape(-1, Co).sum(0), 2e-3, "sum " + tag)
            close(s[1], ref_pre.reshape(-1, Co).pow(2).sum(0), 2e-3, "sumsq " + tag)
            if splits > 1:
                y2, st2 = h.conv2d_same(x, wp, Co, act="lrelu", stats=True, cfg=cfg, bkn=bool(bkn), splits=splits)
                assert torch.equal(y, y2) and torch.equal(st, st2), "nondeterministic " + tag


# ping-pong K loop (240..259) and the deep rings (NS 4 / 5: 220..239, whose tail waits were once
# wrong): split counts that give every k-split length from 1 to 6 and the full 50 k-tiles
DEEP = [220, 223, 225, 226, 230, 233, 235]
PP = [246, 247, 256, 257, 258]
SPLITS_TAIL = (1, 9, 10, 13, 17, 25, 50)


@pytest.mark.parametrize("bkn", [0, 1])
@pytest.mark.parametrize("cfg", DEEP + PP)
def test_igemm3_pipeline_tails(cfg, bkn):
    """Pipeline prologue / tail of the deep-ring and ping-pong K loops: every number of k-tiles
    per split from 1 to NS + 1 (and 50), both weight layouts, fused lrelu + BN statistics,
    against the fp32 reference; split results bitwise reproducible."""
    h = H()
    B, Hs, Ci, Co = 4, 16, 128, 256
    if h.igemm3_lds(cfg) > 160 * 1024:
        pytest.skip("tile does not fit the LDS at this depth")
    x = bf(rnd(B, Hs, Hs, Ci, seed=140))
    w = bf(rnd(5, 5, Ci, Co, scale=0.05, seed=141))
    wt = h.pack_conv_weight(w.float(), "conv", "fwd")
    ref_pre = R.conv2d_same(x.float(), w.float())
    wp = w.reshape(25, Ci, Co).contiguous() if bkn else wt
    for splits in SPLITS_TAIL:
        y, st = h.conv2d_same(x, wp, Co, act="lrelu", stats=True, cfg=cfg, bkn=bool(bkn), splits=splits)
        tag = "cfg%d bkn%d s%d" % (cfg, bkn, splits)
        close(y, R.lrelu(ref_pre), 1.5e-2, tag)
        s = st.sum(0)
        close(s[0], ref_pre.reshape(-1, Co).sum(0), 2e-3, "sum " + tag)
        close(s[1], ref_pre.reshape(-1, Co).pow(2).sum(0), 2e-3, "sumsq " + tag)
        y2, st2 = h.conv2d_same(x, wp, Co, act="lrelu", stats=True, cfg=cfg, bkn=bool(bkn), splits=splits)
        assert torch.equal(y, y2) and torch.equal(st, st2), "nondeterministic " + tag


@pytest.mark.parametrize("cfg", PP)
def test_igemm3_pingpong_deconv_dgrad_bnb(cfg):
    """Ping-pong K loop on the other GEMMs of the step: the 4-phase transposed conv (9/6/6/4 taps),
    the G data gradient (k-major weight) and the fused BN-backward statistics store pass."""
    h = H()
    B, Hi, Ho, Ci, Co = 8, 8, 16, 128, 128
    x = bf(rnd(B, Hi, Hi, Ci, seed=142))
    w = bf(rnd(5, 5, Co, Ci, scale=0.05, seed=143))
    bias = rnd(Co, scale=0.1, seed=144)
    ref = R.conv2d_transpose_same(x.float(), w.float(), (Ho, Ho), bias)
    for splits in (1, 2, 5):
        y = h.conv2d_transpose_same(x, w.reshape(25, Co, Ci), Co, (Ho, Ho), bias=bias, out_f32=True, cfg=cfg,
                                    splits=splits)
        close(y, ref, 2e-3, "deconv cfg%d s%d" % (cfg, splits))
    xd = rnd(B, Hi, Hi, Ci, seed=145).requires_grad_(True)
    yd = R.conv2d_transpose_same(xd, w.float(), (Ho, Ho))
    dy = bf(rnd(B, Ho, Ho, Co, seed=146))
    (gx,) = torch.autograd.grad(yd, xd, dy.float())
    for splits in (1, 4):
        out = h.conv2d_same(dy, w.reshape(25, Co, Ci), Ci, out_f32=True, cfg=cfg, bkn=True, splits=splits)
        close(out, gx, 2e-3, "G dgrad cfg%d s%d" % (cfg, splits))
    test_igemm_fused_bn_backward_stats(cfg)


@pytest.mark.parametrize("B,Hi,Ho,Ci,Co", [(8, 4, 8, 256, 128), (2, 4, 7, 64, 64), (4, 8, 16, 128, 64)])
def test_igemm3_deconv_and_dgrad_layouts(B, Hi, Ho, Ci, Co):
    h = H()
    x = bf(rnd(B, Hi, Hi, Ci, seed=42))
    w = bf(rnd(5, 5, Co, Ci, scale=0.05, seed=43))  # deconv [5,5,out,in] = [25][N][Kc] (bt layout)
    bias = rnd(Co, scale=0.1, seed=44)
    ref = R.conv2d_transpose_same(x.float(), w.float(), (Ho, Ho), bias)
    for cfg in (200, 203, 205, 212, 215, 206, 217, 218):
        for splits in (1, 2, 5):
            y = h.conv2d_transpose_same(x, w.reshape(25, Co, Ci), Co, (Ho, Ho), bias=bias, out_f32=True, cfg=cfg,
                                        splits=splits)
            close(y, ref, 2e-3, "deconv cfg%d s%d" % (cfg, splits))
    # G dgrad = conv of dy with the deconv weight read k-major ([25][Kc=out][N=in], bkn)
    xd = rnd(B, Hi, Hi, Ci, seed=45).requires_grad_(True)
    yd = R.conv2d_transpose_same(xd, w.float(), (Ho, Ho))
    dy = bf(rnd(B, Ho, Ho, Co, seed=46))
    (gx,) = torch.autograd.grad(yd, xd, dy.float())
    for cfg in (200, 205, 213, 216, 207):
        for splits in (1, 4):
            out = h.conv2d_same(dy, w.reshape(25, Co, Ci), Ci, out_f32=True, cfg=cfg, bkn=True, splits=splits)
            close(out, gx, 2e-3, "G dgrad cfg%d s%d" % (cfg, splits))


HALO = [300, 303, 304, 305, 310, 313, 314, 315]


@pytest.mark.parametrize("B,Hi,Ci,Co", [(8, 4, 512, 256), (4, 8, 256, 128), (2, 16, 128, 64), (1, 32, 64, 64),
                                        (2, 32, 128, 128)])
def test_igemm3_halo_deconv(B, Hi, Ci, Co):
    """Halo K loop (input window of a phase tile staged once per 64-channel chunk, taps read it at
    their shift): the 64x64 ladder's deconv shapes (whole images per tile at 4x4 / 8x8, whole rows
    at 16x16 / 32x32), every halo tile / ring depth that takes the shape, split-K over chunks,
    bias, against the fp32 reference; splits bitwise reproducible; shapes whose window does not
    fit are refused by both the Python policy and the C++ check."""
    h = H()
    Ho = 2 * Hi
    x = bf(rnd(B, Hi, Hi, Ci, seed=242))
    w = bf(rnd(5, 5, Co, Ci, scale=0.05, seed=243))
    bias = rnd(Co, scale=0.1, seed=244)
    ref = R.conv2d_transpose_same(x.float(), w.float(), (Ho, Ho), bias)
    ran = 0
    for cfg in HALO:
        for splits in (1, 2, 4):
            ok = h.halo_ok(cfg, 1, B, Ho, Ho, Ci, False, splits)
            if not ok:
                if splits == 1:
                    with pytest.raises(RuntimeError):
                        h.conv2d_transpose_same(x, w.reshape(25, Co, Ci), Co, (Ho, Ho), bias=bias, out_f32=True,
                                                cfg=cfg, splits=splits)
                continue
            y = h.conv2d_transpose_same(x, w.reshape(25, Co, Ci), Co, (Ho, Ho), bias=bias, out_f32=True, cfg=cfg,
                                        splits=splits)
            close(y, ref, 2e-3, "halo deconv cfg%d s%d" % (cfg, splits))
            if splits > 1:
                y2 = h.conv2d_transpose_same(x, w.reshape(25, Co, Ci), Co, (Ho, Ho), bias=bias, out_f32=True, cfg=cfg,
                                             splits=splits)
                assert torch.equal(y, y2), "nondeterministic cfg%d s%d" % (cfg, splits)
            ran += 1
    assert ran >= 4


@pytest.mark.parametrize("cfg", [303, 305, 313, 315])
def test_igemm3_halo_bn_backward_stats(cfg):
    """The halo K loop feeding the fused BN-backward statistics store pass (D's data gradients);
    its chunk-major k order rounds differently from the tap-major loops, so the stored gradient is
    compared with the same cfg's plain GEMM."""
    test_igemm_fused_bn_backward_stats(cfg, ref_cfg=cfg)


@pytest.mark.parametrize("cfg", [200, 211, 213, 206, 216, 217, 218])
def test_igemm_fused_bn_backward_stats(cfg, ref_cfg=200):
    """Data-gradient GEMM with the BN-backward statistics fused into its store pass (epilogue.h
    vec_store_bnb): stored dL/da == the plain GEMM's, partials sum to (sum g, sum g * xhat) with
    g = dL/da * lrelu'(y), for 4- and 8-wave igemm3 tiles."""
    h = H()
    B, Hi, Ci, Co = 4, 16, 128, 64
    Ho = 2 * Hi
    dy = bf(rnd(B, Hi, Hi, Ci, seed=60))
    w = bf(rnd(5, 5, Co, Ci, scale=0.05, seed=61)).reshape(25, Co, Ci).contiguous()
    x = bf(rnd(B, Ho, Ho, Co, seed=62))
    y = bf(rnd(B, Ho, Ho, Co, seed=63) - 0.3)
    mean = rnd(1, Co, scale=0.2, seed=64)
    rstd = rnd(1, Co, seed=65).abs() + 0.5
    if not h.bnb_fits(cfg):
        pytest.skip("tile has no LDS for the fused statistics")
    bm = h.tile_of(cfg)[0]
    mph = B * Hi * Hi
    da_ref = h.conv2d_transpose_same(dy, w, Co, (Ho, Ho), cfg=ref_cfg)
    da = torch.empty_like(da_ref)
    mt = -(-mph // bm)
    st = torch.empty(mt * 4, 2, Co, device=dev)
    prog = h.ext().Program()
    prog.igemm_ex("bnb", 1, h._p(dy), h._p(w), h._p(da), B, Hi, Hi, Ci, Ho, Ho, Co, 1, 1, cfg, 0, Co, 0, 0, 0, 0.2,
                  h._p(st), 0, 0, -1, 1, h._p(x), h._p(y), h._p(mean), h._p(rstd), mph, 2, 0.2, 0)
    h.run(prog)
    torch.cuda.synchronize()
    assert torch.equal(da, da_ref)
    g = da.float() * torch.where(y.float() > 0, 1.0, 0.2)
    xh = (x.float() - mean.reshape(Co)) * rstd.reshape(Co)
    s = st.sum(0)
    close(s[0], g.reshape(-1, Co).sum(0), 2e-3, "sum g cfg%d" % cfg)
    close(s[1], (g * xh).reshape(-1, Co).sum(0), 2e-3, "sum g xhat cfg%d" % cfg)


def test_igemm3_plain_im2col_bkn():
    """3-channel layers: im2col rows [M][80] x the natural weight [75][N] (rows 75..79 -> 0)."""
    h = H()
    B, Hs, C, Co = 4, 64, 3, 64
    x = bf(rnd(B, Hs, Hs, C, seed=47))
    col = h.im2col_s2(x, 80)
    w = bf(rnd(5, 5, C, Co, scale=0.05, seed=48))
    ref = R.conv2d_same(x.float(), w.float()).reshape(-1, Co)
    for cfg in (201, 203, 205, 211):
        y = h.gemm_plain(col, w.reshape(75, Co).contiguous(), out_f32=True, cfg=cfg, bkn=True)
        close(y, ref, 2e-3, "im2col bkn cfg%d" % cfg)


def test_wgrad_conv_and_deconv():
    h = H()
    B, Hs, Ci, Co = 4, 16, 64, 128
    x = bf(rnd(B, Hs, Hs, Ci, seed=17))
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=18).requires_grad_(True)
    dy = bf(rnd(B, 8, 8, Co, seed=19))
    y = R.conv2d_same(x.float(), w)
    (gw,) = torch.autograd.grad(y, w, dy.float())
    out = h.conv_wgrad(x, dy, pad=1)
    close(out.reshape(5, 5, Ci, Co), gw, 2e-3, "conv wgrad")
    for cfg in h.WGRAD_CFGS:
        out = h.conv_wgrad(x, dy, pad=1, cfg=cfg, splits=3)
        close(out.reshape(5, 5, Ci, Co), gw, 2e-3, "conv wgrad cfg%d" % cfg)
    # deconv: Y = deconv(X), W [5,5,co,ci]; G-operand = dY (gathered), Dm = X
    Xd = bf(rnd(B, 8, 8, Ci, seed=20))
    wd = rnd(5, 5, Co, Ci, scale=0.05, seed=21).requires_grad_(True)
    yd = R.conv2d_transpose_same(Xd.float(), wd, (Hs, Hs))
    dyd = bf(rnd(B, Hs, Hs, Co, seed=22))
    (gwd,) = torch.autograd.grad(yd, wd, dyd.float())
    outd = h.conv_wgrad(dyd, Xd, pad=1)
    close(outd.reshape(5, 5, Co, Ci), gwd, 2e-3, "deconv wgrad")


@pytest.mark.parametrize("cfg,B,Hs,Ci,Co", [(400, 4, 32, 64, 128), (401, 3, 32, 64, 64), (402, 4, 16, 64, 64),
                                            (403, 2, 64, 64, 64), (404, 2, 16, 128, 128), (405, 2, 32, 128, 64),
                                            (406, 2, 16, 128, 80), (407, 2, 32, 128, 32), (410, 4, 32, 64, 128),
                                            (414, 2, 16, 128, 128), (416, 2, 16, 128, 80),
                                            (412, 2, 16, 128, 128), (410, 2, 32, 192, 64), (418, 2, 128, 64, 64),
                                            (419, 8, 8, 256, 128), (409, 4, 8, 64, 64)])
def test_wgrad5_halo_rows_conv_and_deconv(cfg, B, Hs, Ci, Co):
    """wgrad5.hip (a kernel row of 5 taps per workgroup, the input rows staged once as a window)
    vs autograd: every configuration, split-K 1/3/5 (uneven and empty-tail splits), a partial last
    channel block (Nc = 80 over 32-wide blocks), conv and deconv operand roles; a second launch of
    the recorded op gives the same bits (split counters re-armed)."""
    h = H()
    Ho = Hs // 2
    pad = (max((Ho - 1) * 2 + 5 - Hs, 0)) // 2
    x = bf(rnd(B, Hs, Hs, Ci, seed=180))
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=181).requires_grad_(True)
    dy = bf(rnd(B, Ho, Ho, Co, seed=182))
    (gw,) = torch.autograd.grad(R.conv2d_same(x.float(), w), w, dy.float())
    for sp in (1, 3, 5):
        out = h.conv_wgrad3(x, dy, pad, cfg=cfg, splits=sp, scale=0.5)
        close(out.reshape(5, 5, Ci, Co), 0.5 * gw, 2e-3, "conv wgrad5 cfg%d sp%d" % (cfg, sp))
    if Co == Ci:  # deconv roles: G-operand = dY (Co = Mc channels, gathered), Dm = X
        Xd = bf(rnd(B, Ho, Ho, Ci, seed=183))
        wd = rnd(5, 5, Co, Ci, scale=0.05, seed=184).requires_grad_(True)
        yd = R.conv2d_transpose_same(Xd.float(), wd, (Hs, Hs))
        dyd = bf(rnd(B, Hs, Hs, Co, seed=185))
        (gwd,) = torch.autograd.grad(yd, wd, dyd.float())
        outd = h.conv_wgrad3(dyd, Xd, pad, cfg=cfg, splits=4)
        close(outd.reshape(5, 5, Co, Ci), gwd, 2e-3, "deconv wgrad5 cfg%d" % cfg)
    prog = h.ext().Program()
    o = torch.empty(25, Ci, Co, device=dev)
    prog.wgrad3("w5", h._p(x), Hs, Hs, Ci, h._p(dy), B, Ho, Ho, Co, pad, cfg, 3, h._p(o), 1.0, 0)
    h.run(prog)
    first = o.clone()
    h.run(prog)
    assert torch.equal(first, o)


@pytest.mark.parametrize("cfg,B,Hs,Ci,Co", [(410, 4, 32, 64, 128), (413, 2, 64, 64, 64), (418, 2, 128, 64, 64),
                                            (412, 2, 16, 128, 128)])
def test_wgrad5_fp16(cfg, B, Hs, Ci, Co):
    """wgrad5.hip's fp16 build (the 256x256 fp16 step runs it) vs autograd, split-K 1 and 5."""
    h = H()
    Ho = Hs // 2
    pad = (max((Ho - 1) * 2 + 5 - Hs, 0)) // 2
    x = rnd(B, Hs, Hs, Ci, seed=190).to(torch.float16).contiguous()
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=191).requires_grad_(True)
    dy = rnd(B, Ho, Ho, Co, seed=192).to(torch.float16).contiguous()
    (gw,) = torch.autograd.grad(R.conv2d_same(x.float(), w), w, dy.float())
    for sp in (1, 5):
        out = h.conv_wgrad3(x, dy, pad, cfg=cfg, splits=sp)
        close(out.reshape(5, 5, Ci, Co), gw, 2e-3, "fp16 conv wgrad5 cfg%d sp%d" % (cfg, sp))


@pytest.mark.parametrize("B,Hs,Ci,Co", [(4, 16, 64, 128), (2, 8, 128, 256), (3, 7, 64, 64), (2, 14, 256, 128)])
def test_wgrad3_conv_and_deconv_all_tiles(B, Hs, Ci, Co):
    """wgrad3.hip (LDS-DMA pipeline, in-kernel split-K) vs autograd: every tile x LDS-stage
    config, split-K 1/3/4 (uneven splits, empty-tail splits), conv and deconv operand roles,
    odd spatial sizes; a second launch of the same recorded op gives the same bits."""
    h = H()
    Ho = -(-Hs // 2)
    pad = (max((Ho - 1) * 2 + 5 - Hs, 0)) // 2
    x = bf(rnd(B, Hs, Hs, Ci, seed=80))
    w = rnd(5, 5, Ci, Co, scale=0.05, seed=81).requires_grad_(True)
    dy = bf(rnd(B, Ho, Ho, Co, seed=82))
    (gw,) = torch.autograd.grad(R.conv2d_same(x.float(), w), w, dy.float())
    for cfg in (300, 301, 302, 303, 310, 311, 312, 313, 320, 322, 330, 332):
        bm, bn = h.WGRAD3_TILES[cfg % 10]
        if cfg >= 320 and 2 * Ci != bm:  # two-tap tiles: BM = 2 Mc
            continue
        for sp in (1, 3, 4):
            out = h.conv_wgrad3(x, dy, pad, cfg=cfg, splits=sp, scale=0.5)
            close(out.reshape(5, 5, Ci, Co), 0.5 * gw, 2e-3, "conv wgrad3 cfg%d sp%d" % (cfg, sp))
    # deconv: Y = deconv(X) [B,Hs,Hs,Co] from X [B,Ho,Ho,Ci]; G-operand = dY (gathered), Dm = X
    Xd = bf(rnd(B, Ho, Ho, Ci, seed=83))
    wd = rnd(5, 5, Co, Ci, scale=0.05, seed=84).requires_grad_(True)
    yd = R.conv2d_transpose_same(Xd.float(), wd, (Hs, Hs))
    dyd = bf(rnd(B, Hs, Hs, Co, seed=85))
    (gwd,) = torch.autograd.grad(yd, wd, dyd.float())
    for cfg in (300, 313):
        outd = h.conv_wgrad3(dyd, Xd, pad, cfg=cfg, splits=4)
        close(outd.reshape(5, 5, Co, Ci), gwd, 2e-3, "deconv wgrad3 cfg%d" % cfg)
    # replay determinism (split-K counters re-armed by the kernel)
    prog = h.ext().Program()
    out = torch.empty(25, Ci, Co, device=dev)
    prog.wgrad3("w3", h._p(x), Hs, Hs, Ci, h._p(dy), B, Ho, Ho, Co, pad, 300, 4, h._p(out), 1.0, 0)
    h.run(prog)
    first = out.clone()
    h.run(prog)
    torch.cuda.synchronize()
    assert torch.equal(first, out)


def test_wgrad_plain_im2col():
    h = H()
    B, Hs, C, Co = 4, 32, 3, 64
    x = bf(rnd(B, Hs, Hs, C, seed=23))
    w = rnd(5, 5, C, Co, scale=0.05, seed=24).requires_grad_(True)
    dy = bf(rnd(B, Hs // 2, Hs // 2, Co, seed=25))
    (gw,) = torch.autograd.grad(R.conv2d_same(x.float(), w), w, dy.float())
    col = h.im2col_s2(x, 80)
    out = h.conv_wgrad(col, dy.reshape(-1, Co), pad=0, mode=2)
    close(out[:75].reshape(5, 5, C, Co), gw, 2e-3, "plain wgrad")


def _prog():
    return H().ext().Program()


def _p(t):
    return 0 if t is None else t.data_ptr()


def test_bn_forward_backward_groups():
    """colstats -> finalize (+EMA) -> apply(act) and the backward chain vs autograd (2 groups)."""
    h = H()
    groups, Bg, Hs, C = 2, 4, 8, 128
    R_ = groups * Bg * Hs * Hs
    x = bf(rnd(groups * Bg, Hs, Hs, C, scale=2.0, seed=26) + 0.3)
    gamma = (1 + 0.1 * rnd(C, seed=27)).contiguous()
    beta = (0.1 * rnd(C, seed=28)).contiguous()
    rows_pb = 64
    P = R_ // rows_pb
    part = torch.empty(P, 2, C, device=dev)
    mean = torch.empty(groups, C, device=dev)
    rstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    ema_m = torch.zeros(groups, C, device=dev)
    ema_v = torch.zeros(groups, C, device=dev)
    y = torch.empty_like(x)
    pr = _prog()
    pr.colstats("st", 0, _p(x), 0, 0, 0, 0, 0, 0.2, R_, C, rows_pb, R_ // groups, _p(part), 0)
    pr.bn_finalize("fin", _p(part), P // groups, groups, C, float(R_ // groups), _p(gamma), _p(beta), 1e-5,
                   _p(mean), _p(rstd), _p(scale), _p(shift), _p(ema_m), _p(ema_v), 0.9, 0)
    pr.bn_apply_act("apply", _p(x), _p(y), _p(scale), _p(shift), R_, C, R_ // groups, 2, 0.2, 0)
    h.run(pr)
    xr = x.float().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    m_ref, v_ref = R.moments(xr, groups)
    yr = R.lrelu(R.batch_norm(xr, m_ref, v_ref, br, gr, 1e-5, groups=groups))
    close(mean, m_ref, 1e-4, "mean")
    close(1.0 / rstd ** 2 - 1e-5, v_ref, 1e-3, "var")
    close(ema_m, 0.1 * m_ref, 1e-4, "ema mean")
    close(y, yr, 1.5e-2, "bn apply")
    # backward
    dy = bf(rnd(groups * Bg, Hs, Hs, C, seed=29))
    gx, gg, gb = torch.autograd.grad(yr, [xr, gr, br], dy.float())
    part2 = torch.empty(P, 2, C, device=dev)
    coef = torch.empty(groups, C, 3, device=dev)
    dgam = torch.empty(C, device=dev)
    dbet = torch.empty(C, device=dev)
    dx = torch.empty_like(x)
    pr = _prog()
    pr.colstats("bst", 1, _p(x), _p(dy), _p(y), _p(mean), _p(rstd), 2, 0.2, R_, C, rows_pb, R_ // groups,
                _p(part2), 0)
    pr.bn_bwd_finalize("bfin", _p(part2), P // groups, groups, C, float(R_ // groups), _p(gamma), _p(mean),
                       _p(rstd), _p(dgam), _p(dbet), _p(coef), 0)
    pr.bn_bwd_apply("bapp", _p(dy), _p(y), _p(x), _p(coef), _p(dx), R_, C, R_ // groups, 2, 0.2, 0)
    h.run(pr)
    close(dgam, gg, 2e-2, "dgamma")
    close(dbet, gb, 2e-2, "dbeta")
    close(dx, gx, 3e-2, "dx")


def test_adam_matches_tf_formula():
    h = H()
    n = 10000 + 3
    w = rnd(n, seed=30)
    g = rnd(n, scale=1e-2, seed=31)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    powers = torch.tensor([0.5, 0.999], device=dev)
    wr, mr, vr = w.clone().cpu(), m.clone().cpu(), v.clone().cpu()
    b1p, b2p = 0.5, 0.999
    for _ in range(3):
        h.adam_(w, g, m, v, powers, 2e-4, 0.5, 0.999, 1e-8)
        R.tf_adam_update(wr, g.cpu(), mr, vr, b1p, b2p, 2e-4, 0.5)
        b1p *= 0.5
        b2p *= 0.999
    assert torch.allclose(w.cpu(), wr, atol=1e-6, rtol=1e-5)
    assert torch.allclose(powers.cpu(), torch.tensor([b1p, b2p]), rtol=1e-6)


def test_gan_loss_kernel():
    h = H()
    B = 37
    logits = rnd(2 * B, scale=4.0, seed=32)
    out = torch.empty(4, device=dev)
    dld = torch.empty(2 * B, device=dev)
    dlg = torch.empty(B, device=dev)
    prob = torch.empty(2 * B, device=dev)
    pr = _prog()
    pr.gan_loss("loss", _p(logits), B, _p(out), _p(dld), _p(dlg), _p(prob), 0)
    h.run(pr)
    lr = logits[:B].clone().requires_grad_(True)
    lf = logits[B:].clone().requires_grad_(True)
    dr, df, gl, dl = R.gan_losses(lr, lf)
    close(out, torch.stack([dr, df, gl, dl]), 1e-5, "losses")
    gdr, gdf = torch.autograd.grad(dl, [lr, lf], retain_graph=True)
    (ggf,) = torch.autograd.grad(gl, [lf])
    close(dld, torch.cat([gdr, gdf]), 1e-5, "dl_d")
    close(dlg, ggf, 1e-5, "dl_g")


def test_linear_and_head():
    h = H()
    B, K, N = 33, 100, 8192
    z = rnd(B, K, seed=33)
    W = rnd(K, N, scale=0.02, seed=34)
    b = rnd(N, scale=0.1, seed=35)
    out = torch.empty(B, N, device=dev, dtype=torch.bfloat16)
    dh = bf(rnd(B, N, seed=36))
    dW = torch.empty(K, N, device=dev)
    db = torch.empty(N, device=dev)
    pr = _prog()
    pr.linear_fwd("lin", _p(z), _p(W), _p(b), _p(out), B, K, N, 0)
    pr.linear_wgrad("linw", _p(z), _p(dh), _p(dW), _p(db), B, K, N, 0)
    h.run(pr)
    close(out, z @ W + b, 1e-2, "linear fwd")
    close(dW, z.t() @ dh.float(), 1e-3, "linear wgrad")
    close(db, dh.float().sum(0), 1e-3, "linear bias grad")
    # fused BN partial statistics (channel = column % C; partial row = (8-row block, column // C))
    C = 512
    part = torch.full((-(-B // 8) * (N // C), 2, C), float("nan"), device=dev)
    out2 = torch.empty_like(out)
    pr = _prog()
    pr.linear_fwd("lin", _p(z), _p(W), _p(b), _p(out2), B, K, N, 0, _p(part), C)
    h.run(pr)
    assert torch.equal(out2, out)
    o = out.float().reshape(B, N // C, C)
    close(part[:, 0].sum(0), o.sum((0, 1)), 1e-5, "linear stats sum")
    close(part[:, 1].sum(0), (o * o).sum((0, 1)), 1e-5, "linear stats sumsq")
    ob = torch.nn.functional.pad(o, (0, 0, 0, 0, 0, 40 - B)).reshape(5, 8, N // C, C).sum(1).reshape(-1, C)
    close(part[:, 0], ob, 1e-5, "linear stats per block")
    # z generated inside the kernel == philox_uniform + linear (bit-identical z and output)
    step = torch.tensor([7], dtype=torch.int64, device=dev)
    z1, z2 = torch.empty(B, K, device=dev), torch.full((B, K), float("nan"), device=dev)
    o1, o2 = torch.empty_like(out), torch.empty_like(out)
    pr = _prog()
    pr.philox_uniform("z", _p(z1), z1.numel(), 123457, _p(step), 0, -1.0, 1.0, 0)
    pr.linear_fwd("lin", _p(z1), _p(W), _p(b), _p(o1), B, K, N, 0)
    pr.linear_fwd("lin_gen", _p(z2), _p(W), _p(b), _p(o2), B, K, N, 0, 0, 0, _p(step), 123457)
    h.run(pr)
    assert torch.equal(z1, z2) and torch.equal(o1, o2)
    # D head
    R_, Kh = 2 * B, 8192
    x = bf(rnd(R_, Kh, seed=37))
    w = rnd(Kh, scale=0.02, seed=38)
    hb = rnd(1, seed=39)
    logit = torch.empty(R_, device=dev)
    dl = rnd(R_, seed=40)
    dx = torch.empty(R_, Kh, device=dev, dtype=torch.bfloat16)
    part = torch.empty(8, Kh, device=dev)
    dw = torch.empty(Kh, device=dev)
    dbh = torch.empty(1, device=dev)
    pr = _prog()
    pr.gemv_head("head", _p(x), _p(w), _p(hb), _p(logit), R_, Kh, 0)
    pr.head_dgrad("hd", _p(dl), _p(w), _p(dx), R_, Kh, 0)
    pr.head_wgrad("hw", _p(x), _p(dl), _p(part), R_, Kh, 8, _p(dw), _p(dbh), 0)
    h.run(pr)
    close(logit, x.float() @ w + hb, 1e-4, "head fwd")
    close(dx, dl[:, None] * w[None, :], 1e-2, "head dgrad")
    close(dw, x.float().t() @ dl, 1e-4, "head wgrad")
    close(dbh, dl.sum().reshape(1), 1e-5, "head bias")


def test_philox_uniform_range_and_determinism():
    h = H()
    n = 128 * 100
    out1 = torch.empty(n, device=dev)
    out2 = torch.empty(n, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    pr = _prog()
    pr.philox_uniform("z", _p(out1), n, 1234, _p(step), 0, -1.0, 1.0, 0)
    pr.philox_uniform("z", _p(out2), n, 1234, _p(step), 0, -1.0, 1.0, 0)
    h.run(pr)
    assert torch.equal(out1, out2)
    assert out1.min() >= -1 and out1.max() < 1
    assert abs(out1.mean().item()) < 0.03 and abs(out1.std().item() - 1 / math.sqrt(3)) < 0.02


@pytest.mark.parametrize("B,Hi,Ho,C,N,dtype", [(4, 32, 64, 64, 3, "bf16"), (2, 4, 7, 64, 3, "bf16"),
                                                (3, 14, 28, 64, 1, "bf16"), (2, 16, 32, 128, 3, "fp16"),
                                                (2, 16, 32, 64, 3, "fp16"), (2, 9, 17, 64, 4, "bf16")])
def test_narrow_deconv(B, Hi, Ho, C, N, dtype):
    """Direct conv_transpose for N <= 4 outputs (G's RGB layer, D layer-0 data gradient): the
    MFMA kernel (C = 64) and the v_dot2 VALU kernel (other C): bias + tanh, odd sizes (pad 2),
    1 and 4 channels, fp16 build."""
    h = H()
    edt = torch.float16 if dtype == "fp16" else torch.bfloat16
    x = rnd(B, Hi, Hi, C, seed=60).to(edt)
    w = (rnd(5, 5, N, C, scale=0.05, seed=61)).to(edt)
    bias = rnd(N, scale=0.1, seed=62)
    y = h.narrow_deconv(x, w, (Ho, Ho), bias=bias, act="tanh")
    ref = torch.tanh(R.conv2d_transpose_same(x.float(), w.float(), (Ho, Ho), bias))
    close(y, ref, 1e-2, "narrow deconv")
    # as the data gradient of a conv with HWIO weight [5,5,N,C]
    xg = rnd(B, Ho, Ho, N, seed=63).requires_grad_(True)
    yc = R.conv2d_same(xg, w.float())
    (gx,) = torch.autograd.grad(yc, xg, x.float())
    close(h.narrow_deconv(x, w, (Ho, Ho)), gx, 1e-2, "narrow as conv dgrad")


@pytest.mark.parametrize("B,Hi,Ho,N", [(4, 32, 64, 3), (3, 14, 28, 1), (2, 9, 17, 4)])
def test_narrow_deconv_dact(B, Hi, Ho, N):
    """The image gradient with G's tanh backward fused: y = conv_transpose(x, w) * (1 - ya^2)
    and the bias gradient sum(y) over every pixel (per-workgroup partials + sliced sum)."""
    h = H()
    x = bf(rnd(B, Hi, Hi, 64, seed=64))
    w = bf(rnd(5, 5, N, 64, scale=0.05, seed=65))
    ya = bf(torch.tanh(rnd(B, Ho, Ho, N, scale=2.0, seed=66)))
    y = torch.empty(B, Ho, Ho, N, device=dev, dtype=torch.bfloat16)
    db = torch.empty(N, device=dev)
    prog = h.ext().Program()
    pad = max((Hi - 1) * 2 + 5 - Ho, 0) // 2
    prog.narrow_deconv_dact("nd", h._p(x), h._p(w), h._p(y), h._p(ya), B, Hi, Hi, 64, Ho, Ho, N, pad, 3, 0.0,
                            h._p(db), 0)
    h.run(prog)
    torch.cuda.synchronize()
    ref = R.conv2d_transpose_same(x.float(), w.float(), (Ho, Ho)) * (1 - ya.float() ** 2)
    close(y, ref, 1e-2, "narrow deconv dact")
    close(db, y.float().reshape(-1, N).sum(0), 1e-4, "dbias of the stored values")


@pytest.mark.parametrize("B,Hh,C,dtype", [(4, 64, 3, "bf16"), (2, 28, 1, "bf16"), (3, 33, 4, "bf16"),
                                          (2, 64, 3, "fp16"), (1, 7, 3, "bf16"), (2, 128, 3, "bf16"),
                                          (80, 64, 3, "bf16")])
def test_nconv(B, Hh, C, dtype):
    """narrow2.hip nconv (persistent, Cin <= 4 -> 64, + bias + lrelu) vs the fp32 TF-SAME oracle:
    RGB / gray / 4-channel, odd sizes (partial tiles, pad 2 at 7 and 33), two column tiles
    (128 -> 64 wide), more tiles than workgroups (80 images: the persistent loop), fp16 build."""
    h = H()
    edt = torch.float16 if dtype == "fp16" else torch.bfloat16
    x = rnd(B, Hh, Hh, C, seed=70).to(edt)
    w = rnd(5, 5, C, 64, scale=0.1, seed=71).to(edt)
    bias = rnd(64, scale=0.1, seed=72)
    y = h.nconv(x, w, bias=bias, act="lrelu")
    ref = R.lrelu(R.conv2d_same(x.float(), w.float(), bias))
    close(y, ref, 1e-2, "nconv")


@pytest.mark.parametrize("B,Hh,act", [(4, 64, "relu"), (3, 33, "lrelu"), (70, 64, "relu")])
def test_nconv_bn_backward_stats(B, Hh, act):
    """nconv as G's RGB-layer data gradient (no bias / act) with the BN-backward statistics of
    the layer below fused: the stored dL/da equals the plain conv; the per-workgroup partials
    sum to (sum g, sum g*xhat), g = dL/da * act'(y), of the stored (rounded) values."""
    h = H()
    Ho = -(-Hh // 2)
    dimg = bf(rnd(B, Hh, Hh, 3, seed=73))
    w = bf(rnd(5, 5, 3, 64, scale=0.1, seed=74))
    x = bf(rnd(B, Ho, Ho, 64, seed=75))
    y = bf(rnd(B, Ho, Ho, 64, seed=76) - 0.3)
    mean = rnd(64, scale=0.2, seed=77)
    rstd = rnd(64, seed=78).abs() + 0.5
    da, part = h.nconv(dimg, w, bnb=(x, y, mean, rstd, act))
    ref = R.conv2d_same(dimg.float(), w.float())
    close(da, ref, 1e-2, "nconv dgrad")
    assert torch.equal(da, h.nconv(dimg, w))
    slope = 0.2 if act == "lrelu" else 0.0
    g = da.float() * torch.where(y.float() > 0, 1.0, slope)
    xh = (x.float() - mean) * rstd
    s = part.sum(0)
    close(s[0], g.reshape(-1, 64).sum(0), 2e-3, "sum g")
    close(s[1], (g * xh).reshape(-1, 64).sum(0), 2e-3, "sum g xhat")


@pytest.mark.parametrize("B,Hh,C,dtype", [(4, 64, 3, "bf16"), (2, 28, 1, "bf16"), (3, 33, 4, "bf16"),
                                          (2, 64, 3, "fp16"), (1, 7, 3, "bf16"), (2, 128, 3, "bf16"),
                                          (40, 64, 3, "bf16"), (2, 256, 3, "fp16"), (1, 256, 3, "bf16")])
def test_nwgrad(B, Hh, C, dtype):
    """narrow2.hip nwgrad vs autograd: the conv role (D layer 0: x = image, d = dL/d(conv out))
    and the deconv role (G's RGB layer: x = dL/d(deconv out), d = the layer input, TF layout
    [5,5,co,ci]); gray / 4-channel, odd sizes, 64-wide outputs (4-row chunks), several chunks
    per workgroup (40 images), fp16; a second launch gives the same bits."""
    h = H()
    edt = torch.float16 if dtype == "fp16" else torch.bfloat16
    Ho = -(-Hh // 2)
    pad = max((Ho - 1) * 2 + 5 - Hh, 0) // 2
    x = rnd(B, Hh, Hh, C, seed=90).to(edt)
    w = rnd(5, 5, C, 64, scale=0.05, seed=91).requires_grad_(True)
    dy = rnd(B, Ho, Ho, 64, seed=92).to(edt)
    (gw,) = torch.autograd.grad(R.conv2d_same(x.float(), w), w, dy.float())
    out = h.nwgrad(x, dy, pad)
    close(out.reshape(5, 5, C, 64), gw, 3e-3, "nwgrad conv")
    assert torch.equal(out, h.nwgrad(x, dy, pad))
    # deconv role: Y = deconv(X) [B,Hh,Hh,C] from X [B,Ho,Ho,64], W [5,5,C,64]
    Xd = rnd(B, Ho, Ho, 64, seed=93).to(edt)
    wd = rnd(5, 5, C, 64, scale=0.05, seed=94).requires_grad_(True)
    dyd = rnd(B, Hh, Hh, C, seed=95).to(edt)
    (gwd,) = torch.autograd.grad(R.conv2d_transpose_same(Xd.float(), wd, (Hh, Hh)), wd, dyd.float())
    close(h.nwgrad(dyd, Xd, pad).reshape(5, 5, C, 64), gwd, 3e-3, "nwgrad deconv")


@pytest.mark.parametrize("P,groups,C", [(2048, 2, 80), (700, 1, 512), (96, 2, 64)])
def test_bn_finalize_split_paths(P, groups, C):
    """Many partial rows -> the sliced finalize with a last-arrival combine (counters reset, so a
    second launch of the same op gives the same bits); compared with float64 sums."""
    h = H()
    ext = h.ext()
    _p = h._p
    g = torch.Generator().manual_seed(70)
    part = (torch.randn(P, 2, C, generator=g, dtype=torch.float64) * 3 + 1).abs()
    part_d = part.float().to(dev)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.rand(C, generator=g) - 0.5).to(dev)
    cnt = 1000.0
    outs = [torch.zeros(groups, C, device=dev) for _ in range(4)]
    ema_m, ema_v = torch.zeros(groups, C, device=dev), torch.zeros(groups, C, device=dev)
    pr = ext.Program()
    pr.bn_finalize("fin", _p(part_d), P // groups, groups, C, cnt, _p(gamma), _p(beta), 1e-5, _p(outs[0]), _p(outs[1]),
                   _p(outs[2]), _p(outs[3]), _p(ema_m), _p(ema_v), 0.9, 0)
    h.run(pr)
    first = [o.clone() for o in outs]
    h.run(pr)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(first, outs)), "second launch differs (counter reset)"
    pg = part.reshape(groups, P // groups, 2, C).sum(1)
    m = pg[:, 0] / cnt
    v = (pg[:, 1] / cnt - m * m).clamp_min(0)
    close(outs[0].cpu(), m, 1e-5, "mean")
    close(outs[1].cpu(), (v + 1e-5).rsqrt(), 1e-4, "rstd")
    # backward coefficients + group-summed dgamma / dbeta
    mean, rstd = outs[0], outs[1]
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    coef = torch.zeros(groups, 3, C, device=dev)
    pr2 = ext.Program()
    pr2.bn_bwd_finalize("bfin", _p(part_d), P // groups, groups, C, cnt, _p(gamma), _p(mean), _p(rstd), _p(dg), _p(db),
                        _p(coef), 0)
    h.run(pr2)
    torch.cuda.synchronize()
    close(db.cpu(), pg[:, 0].sum(0), 1e-5, "dbeta")
    close(dg.cpu(), pg[:, 1].sum(0), 1e-5, "dgamma")
    A = gamma.double().cpu() * rstd.double().cpu()
    close(coef[:, 0].cpu(), A, 1e-5, "coef A")
    close(coef[:, 1].cpu(), -A * pg[:, 1] / cnt * rstd.double().cpu(), 1e-4, "coef x")


@pytest.mark.parametrize("R,C,act", [(256 * 1024, 64, 2), (1000, 64, 1), (128 * 64 * 64, 3, 3), (777, 3, 3),
                                     (4099, 1, 2), (3 * 129, 256, 2), (50, 128, 0)])
def test_act_bwd_dbias(R, C, act):
    """Fused dx = dy * act'(y) + bias gradient (last-arrival reduction): dx bit-exact vs the
    separate act_bwd formula, db vs an fp64 column sum of the stored dx; replay gives the same bits."""
    h = H()
    dy = bf(rnd(R, C, seed=90))
    y = rnd(R, C, seed=91)
    if act == 3:
        y = torch.tanh(y * 2)
    y = bf(y)
    dx, db = h.act_bwd_dbias(dy, y, act, 0.2)
    yf = y.float()
    if act == 1:
        d = (yf > 0).float()
    elif act == 2:
        d = torch.where(yf > 0, torch.ones_like(yf), torch.full_like(yf, 0.2))
    elif act == 3:
        d = 1 - yf * yf
    else:
        d = torch.ones_like(yf)
    ref_dx = (dy.float() * d).to(torch.bfloat16)
    if act == 3:  # 1 - y*y may be contracted into an fma on the GPU: one bf16 ulp
        close(dx, ref_dx, 8e-3, "tanh dx")
    else:
        assert torch.equal(dx, ref_dx)
    ref_db = dx.double().sum(0)
    assert (db.double() - ref_db).abs().max().item() <= 1e-5 * (dx.double().abs().sum(0).max().item() + 1)
    dx2, db2 = h.act_bwd_dbias(dy, y, act, 0.2)
    assert torch.equal(db, db2) and torch.equal(dx, dx2)


@pytest.mark.parametrize("R,K", [(256, 8192), (64, 4096), (10, 200)])
def test_head_bwd_fused(R, K):
    h = H()
    x = bf(rnd(R, K, seed=92))
    dl = rnd(R, seed=93)
    w = rnd(K, scale=0.02, seed=94)
    dx, dW, db = h.head_bwd(x, dl, w)
    close(dW, x.float().t() @ dl, 1e-4, "head dW")
    close(db, dl.sum(0, keepdim=True), 1e-5, "head db")
    assert torch.equal(dx, (dl[:, None] * w[None, :]).to(torch.bfloat16))


@pytest.mark.parametrize("R,groups", [(256, 2), (128, 1)])
def test_head_bwd_bn_stats(R, groups):
    """Head backward with the top BN layer's backward statistics fused in: per (group, spatial
    position) partial rows of (sum g, sum g * xhat), g = dx * lrelu'(y), from the stored dx."""
    h = H()
    K, C = 8192, 512
    S = K // C
    xa = bf(rnd(R, K, seed=95))
    dl = rnd(R, seed=96)
    w = rnd(K, scale=0.02, seed=97)
    bx = bf(rnd(R, K, seed=98))
    by = bf(rnd(R, K, seed=99))
    mean = rnd(groups, C, scale=0.1, seed=100)
    rstd = rnd(groups, C, seed=101).abs() + 0.5
    dx = torch.empty_like(xa)
    dW = torch.empty(K, device=dev)
    db = torch.empty(1, device=dev)
    part = torch.full((groups * S, 2, C), float("nan"), device=dev)
    pr = _prog()
    pr.head_bwd("hb", _p(xa), _p(dl), _p(w), _p(dx), _p(dW), _p(db), R, K, 0, _p(bx), _p(by), _p(mean), _p(rstd), C,
                R // groups, 2, 0.2, _p(part))
    h.run(pr)
    assert torch.equal(dx, (dl[:, None] * w[None, :]).to(torch.bfloat16))
    close(dW, xa.float().t() @ dl, 1e-4, "dW")
    g = dx.float() * torch.where(by.float() > 0, 1.0, 0.2)
    rpg = R // groups
    for gi in range(groups):
        gg = g[gi * rpg:(gi + 1) * rpg].reshape(rpg, S, C)
        xh = (bx.float()[gi * rpg:(gi + 1) * rpg].reshape(rpg, S, C) - mean[gi]) * rstd[gi]
        close(part[gi * S:(gi + 1) * S, 0], gg.sum(0), 1e-4, "sum g")
        close(part[gi * S:(gi + 1) * S, 1], (gg * xh).sum(0), 1e-4, "sum g xhat")


def test_head_gemv_fused_loss_matches_separate():
    """gemv_head with the 3-loss BCE in its last-arriving block == gemv_head + gan_loss (bitwise),
    and replays re-arm the arrival counter."""
    h = H()
    B, K = 64, 8192
    x = bf(rnd(2 * B, K, seed=110))
    w = rnd(K, scale=0.02, seed=111)
    hb = rnd(1, seed=112)
    bufs = [[torch.full((n,), float("nan"), device=dev) for n in (2 * B, 4, 2 * B, B, 2 * B)] for _ in range(2)]
    pr = _prog()
    lg, lo, dd, dg, pb = bufs[0]
    pr.gemv_head("h", _p(x), _p(w), _p(hb), _p(lg), 2 * B, K, 0)
    pr.gan_loss("l", _p(lg), B, _p(lo), _p(dd), _p(dg), _p(pb), 0)
    lg2, lo2, dd2, dg2, pb2 = bufs[1]
    pr.gemv_head("hl", _p(x), _p(w), _p(hb), _p(lg2), 2 * B, K, 0, _p(lo2), _p(dd2), _p(dg2), _p(pb2), 0)
    for _ in range(2):
        h.run(pr)
        torch.cuda.synchronize()
        for a, b in zip(bufs[0], bufs[1]):
            assert torch.equal(a, b)


def test_head_gemv_bn_apply_fused():
    """gemv_head_bn (the top BN layer's apply + LeakyReLU inside the head GEMV, two row groups)
    == bn_apply_act + gemv_head: the written activation bitwise, logits / losses / seeds too."""
    h = H()
    B, K, C = 64, 8192, 512
    x = bf(rnd(2 * B, K, scale=2.0, seed=113))
    w = rnd(K, scale=0.02, seed=114)
    hb = rnd(1, seed=115)
    scale = (1 + 0.2 * rnd(2, C, seed=116)).contiguous()
    shift = (0.2 * rnd(2, C, seed=117)).contiguous()
    ya = torch.empty_like(x)
    yb = torch.empty_like(x)
    bufs = [[torch.full((n,), float("nan"), device=dev) for n in (2 * B, 4, 2 * B, B, 2 * B)] for _ in range(2)]
    pr = _prog()
    lg, lo, dd, dg, pb = bufs[0]
    pr.bn_apply_act("apply", _p(x), _p(ya), _p(scale), _p(shift), 2 * B * (K // C), C, B * (K // C), 2, 0.2, 0)
    pr.gemv_head("hl", _p(ya), _p(w), _p(hb), _p(lg), 2 * B, K, 0, _p(lo), _p(dd), _p(dg), _p(pb), 0)
    lg2, lo2, dd2, dg2, pb2 = bufs[1]
    pr.gemv_head_bn("hbn", _p(x), _p(w), _p(hb), _p(lg2), 2 * B, K, 0, _p(lo2), _p(dd2), _p(dg2), _p(pb2), 0,
                    _p(scale), _p(shift), C, B, 2, 0.2, _p(yb))
    for _ in range(2):
        h.run(pr)
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)  # the activation the backward reads: bitwise
        for a, b in zip(bufs[0], bufs[1]):  # same operands; FMA contraction may differ in the last bit
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,Hi,N", [(4, 32, 3), (3, 16, 1)])
def test_narrow_deconv_bn_input_fused(B, Hi, N):
    """narrow_deconv_bnin (the lower layer's BN apply + ReLU in the halo staging) == bn_apply_act
    + narrow_deconv: the written activation and the RGB output bitwise."""
    h = H()
    Ho = 2 * Hi
    pad = max((Hi - 1) * 2 + 5 - Ho, 0) // 2
    x = bf(rnd(B, Hi, Hi, 64, scale=2.0, seed=120))
    w = bf(rnd(5, 5, N, 64, scale=0.05, seed=121))
    bias = rnd(N, scale=0.1, seed=122)
    scale = (1 + 0.2 * rnd(64, seed=123)).contiguous()
    shift = (0.2 * rnd(64, seed=124)).contiguous()
    a1, a2 = torch.empty_like(x), torch.empty_like(x)
    y1 = torch.empty(B, Ho, Ho, N, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    pr = _prog()
    pr.bn_apply_act("apply", _p(x), _p(a1), _p(scale), _p(shift), B * Hi * Hi, 64, B * Hi * Hi, 1, 0.2, 0)
    pr.narrow_deconv("nd", _p(a1), _p(w), _p(bias), _p(y1), B, Hi, Hi, 64, Ho, Ho, N, pad, 3, 0.2, 0)
    pr.narrow_deconv_bnin("ndb", _p(x), _p(w), _p(bias), _p(y2), B, Hi, Hi, 64, Ho, Ho, N, pad, 3, 0.2, _p(scale),
                          _p(shift), 1, 0.2, _p(a2), 0)
    h.run(pr)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("R,groups,RS", [(256, 2, 4), (128, 1, 4), (256, 2, 2)])
def test_head_bwd_row_splits(R, groups, RS):
    """Head backward with RS row splits: dx bitwise, dW (split partials summed in order by the
    last split of each column block, counters re-armed across launches), per-group BN partial
    rows [(g RS + y) S + sp] summing to the reference statistics."""
    h = H()
    K, C = 8192, 512
    S = K // C
    xa = bf(rnd(R, K, seed=130))
    dl = rnd(R, seed=131)
    w = rnd(K, scale=0.02, seed=132)
    bx = bf(rnd(R, K, seed=133))
    by = bf(rnd(R, K, seed=134))
    mean = rnd(groups, C, scale=0.1, seed=135)
    rstd = rnd(groups, C, seed=136).abs() + 0.5
    dx = torch.empty_like(xa)
    dW = torch.empty(K, device=dev)
    db = torch.empty(1, device=dev)
    part = torch.full((groups * RS * S, 2, C), float("nan"), device=dev)
    pr = _prog()
    pr.head_bwd_rs("hbs", _p(xa), _p(dl), _p(w), _p(dx), _p(dW), _p(db), R, K, 0, _p(bx), _p(by), _p(mean), _p(rstd),
                   C, R // groups, 2, 0.2, _p(part), RS)
    for rep in range(2):
        h.run(pr)
        torch.cuda.synchronize()
        if rep == 0:
            first = dW.clone()
    assert torch.equal(first, dW)
    assert torch.equal(dx, (dl[:, None] * w[None, :]).to(torch.bfloat16))
    close(dW, xa.float().t() @ dl, 1e-4, "dW")
    close(db, dl.sum().reshape(1), 1e-5, "db")
    g = dx.float() * torch.where(by.float() > 0, 1.0, 0.2)
    rpg = R // groups
    ppg = RS * S
    for gi in range(groups):
        gg = g[gi * rpg:(gi + 1) * rpg].reshape(rpg, S, C)
        xh = (bx.float()[gi * rpg:(gi + 1) * rpg].reshape(rpg, S, C) - mean[gi]) * rstd[gi]
        pg = part[gi * ppg:(gi + 1) * ppg].reshape(RS, S, 2, C).sum(0)
        close(pg[:, 0], gg.sum(0), 1e-4, "sum g")
        close(pg[:, 1], (gg * xh).sum(0), 1e-4, "sum g xhat")

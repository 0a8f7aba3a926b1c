"""Loader and thin tensor-level wrappers for the gfx950 kernel library (``_dcgan_hip``).

The extension is built in-tree by ``csrc/build.py`` (``__graft_entry__.build()``). On a
machine with a GPU the HIP path is mandatory: if the extension is missing or was built
for another architecture, :func:`ext` raises instead of silently falling back to PyTorch.

The wrappers below run ONE op through a throw-away ``Program`` on the current torch
stream; they exist for unit tests and for the autograd modules in ``ops.functional``.
The training engine records its whole step into persistent programs instead
(``engine.hip_engine``).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional, Sequence, Tuple

import torch

from ..models.config import same_out, same_pads

_EXT = None

ACT = {None: 0, "none": 0, "relu": 1, "lrelu": 2, "tanh": 3}


class HipUnavailable(RuntimeError):
    pass


def ext():
    """Import the compiled extension (torch must be imported first so that the HIP runtime
    shared by torch and the extension is the one already loaded)."""
    global _EXT
    if _EXT is None:
        try:
            _EXT = importlib.import_module("distributed_tensorflow_for_dcgan_amd._dcgan_hip")
        except ImportError as e:  # pragma: no cover - depends on build state
            raise HipUnavailable(
                "native HIP extension _dcgan_hip is not built; run `python csrc/build.py` "
                "(or __graft_entry__.build()). Original error: %s" % e) from e
    return _EXT


def available() -> bool:
    try:
        ext()
        return torch.cuda.is_available()
    except HipUnavailable:
        return False


def stream_ptr(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def run(prog, streams: Optional[Sequence] = None, begin: int = 0, end: int = -1) -> None:
    if streams is None:
        streams = [torch.cuda.current_stream()]
    prog.run([stream_ptr(s) if not isinstance(s, int) else s for s in streams], begin, end)


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


# --------------------------------------------------------------------------- tile policy
CU_COUNT = 256
IGEMM_CFGS = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (32, 64), 5: (64, 32),
              6: (32, 32), 7: (128, 16), 8: (64, 16), 9: (256, 64)}
IGEMM3_TILES = {0: (128, 128), 1: (256, 64), 2: (64, 256), 3: (128, 64), 4: (64, 128), 5: (64, 64),
                6: (256, 128), 7: (128, 256), 8: (512, 64), 9: (256, 256)}  # 6..9: 8-wave (512-thread) workgroups
IGEMM3_WAVES = {6: 8, 7: 8, 8: 8, 9: 8}
IGEMM3_WM = {0: 2, 1: 4, 2: 1, 3: 2, 4: 2, 5: 2, 6: 4, 7: 2, 8: 8, 9: 4}  # waves along M (igemm3.hip tiles)
# LDS stages of igemm3 cfg 200+10k+id; k = 4, 5 (cfg 240..259): the ping-pong K loop (8-wave tiles,
# conv / deconv modes with Kc % 64 == 0)
IGEMM3_STAGES = (3, 2, 4, 5, 3, 2)


# halo K loop (igemm3.hip PP == 2, cfg 300 + 10 k + id, NS = (3, 2)[k], 4-wave tiles 0 / 3 / 4 / 5):
# deconv phases with the input window of a phase tile staged once per 64-channel chunk
HALO_IDS = (0, 3, 4, 5)
HALO_PIXELS = 224  # window buffer capacity (igemm3.hip HALO_WPW x 4 waves x 8 pixels)


def is_halo(cfg: int) -> bool:
    return 300 <= cfg < 320 and cfg % 10 in HALO_IDS


def igemm3_ns(cfg: int) -> int:
    if cfg >= 300:
        return 3 if cfg < 310 else 2
    return IGEMM3_STAGES[(cfg - 200) // 10]


def halo_ok(cfg: int, mode: int, Bn: int, Hout: int, Wout: int, Kc: int, bkn: bool = False, splits: int = 1) -> bool:
    """Whether a halo cfg can run this GEMM (mirrors csrc/bindings.cpp igemm_ex): a deconv with
    k-contiguous weights, whole 64-channel chunks (split-K over chunks), every phase tile covering
    whole images or whole rows of one image with an input window of <= HALO_PIXELS pixels."""
    if not is_halo(cfg) or mode != 1 or bkn or Kc % 64 or splits > Kc // 64:
        return False
    bm = IGEMM3_TILES[cfg % 10][0]
    for py in (0, 1):
        for px in (0, 1):
            Hq, Wq = (Hout - py + 1) // 2, (Wout - px + 1) // 2
            hw = Hq * Wq
            if hw <= 0:
                continue
            whole, rows = bm % hw == 0, hw % bm == 0 and bm % Wq == 0
            nimg, R = (bm // hw, Hq) if whole else (1, bm // max(1, Wq))
            if not (whole or rows) or nimg * (R + 2) * (Wq + 2) > HALO_PIXELS:
                return False
    return True


def igemm3_pp_ok(cfg: int, mode: int, Kc: int) -> bool:
    """Whether igemm3 cfg can run this GEMM: the ping-pong configs (240..259) need an 8-wave tile
    and whole 64-channel k-tiles of a conv / deconv (no im2col plain mode); the halo configs
    (300..319) are checked with the full geometry by halo_ok."""
    if cfg >= 300:
        return is_halo(cfg) and mode == 1 and Kc % 64 == 0
    if cfg < 240:
        return True
    return cfg % 10 in IGEMM3_WAVES and mode != 2 and Kc % 64 == 0


def igemm3_lds(cfg: int) -> int:
    """Operand-ring bytes of igemm3 cfg (the launch adds room when the epilogue needs more)."""
    bm, bn = IGEMM3_TILES[cfg % 10]
    if cfg >= 300:
        return 2 * HALO_PIXELS * 128 + igemm3_ns(cfg) * bn * 128
    return igemm3_ns(cfg) * (bm + bn) * 128


# fp32 build (igemm_f32.hip): the only tile family of that element type, cfg 200..203
IGEMM_F32_TILES = {200: (64, 64), 201: (128, 64), 202: (64, 16), 203: (128, 128)}


def tile_of(cfg: int, dtype: int = 0) -> Tuple[int, int]:
    """(BM, BN) of an igemm cfg: 0..9 (+100 LDS-DMA) igemm.hip, 200..239 igemm3.hip; dtype 2
    (fp32): igemm_f32.hip; 240..259 igemm3's ping-pong K loop."""
    if dtype == 2:
        return IGEMM_F32_TILES[cfg]
    if cfg >= 200:
        return IGEMM3_TILES[cfg % 10]
    return IGEMM_CFGS[cfg % 100]


def pick_igemm_f32(M: int, N: int, phases: int = 1, rows_per_group: Optional[int] = None,
                   target_blocks: int = 2 * CU_COUNT) -> Optional[Tuple[int, int]]:
    """(cfg, 1) for the fp32 implicit GEMM: the largest tile that still gives ~target_blocks
    workgroups (narrow 64x16 tile for N <= 16, e.g. the RGB layers); no split-K."""
    order = [202] if N <= 16 else ([203, 201, 200] if N >= 128 else [201, 200])
    best = None
    for c in order:
        bm, bn = IGEMM_F32_TILES[c]
        if rows_per_group is not None and rows_per_group % bm:
            continue
        best = c
        if -(-M // bm) * -(-N // bn) * phases >= target_blocks:
            break
    return None if best is None else (best, 1)


def bnb_fits(cfg: int) -> bool:
    """True when the tile's LDS can hold the fused BN-backward statistics scratch (epilogue.h)."""
    bm, bn = tile_of(cfg)
    if cfg < 200:
        return (bm + 8 * bn) * 4 + bm * (bn + 8) * 2 + 16384 <= 2 * (bm + bn) * 128
    nt = 64 * IGEMM3_WAVES.get(cfg % 10, 4)
    wm = IGEMM3_WM[cfg % 10]
    # igemm3: the row-lane scratch may alias the C tile (the store pass has read it by then);
    # (halo tiles have more LDS than this ring estimate, as csrc/bindings.cpp assumes too)
    lds = max(igemm3_ns(cfg) * (bm + bn) * 128, (bm + 2 * wm * bn) * 4 + bm * (bn + 8) * 2)
    return (bm + 2 * wm * bn) * 4 + max(bm * (bn + 8) * 2, 64 * nt) <= lds


WGRAD_CFGS = {0: (128, 128), 1: (64, 128), 2: (128, 64), 3: (64, 64), 4: (32, 64), 5: (64, 32), 6: (32, 32)}


def pick_igemm_cfg(M: int, N: int, phases: int = 1, rows_per_group: Optional[int] = None,
                   target_blocks: int = 2 * CU_COUNT) -> int:
    """Largest tile that still gives >= target_blocks workgroups (fill 256 CUs twice);
    BM must divide rows_per_group when per-group BN statistics are produced."""
    if N <= 16:
        order = [7, 8]
    else:
        order = [0, 1, 2, 3, 4, 5, 6]
    best = None
    for c in order:
        bm, bn = IGEMM_CFGS[c]
        if rows_per_group is not None and rows_per_group % bm != 0:
            continue
        if bn > 16 and N < bn and bn > 32 and c not in (5, 6):
            # avoid tiles wider than N (wasted MFMA columns) unless nothing else fits
            continue
        blocks = -(-M // bm) * -(-N // bn) * phases
        if best is None:
            best = c
        if blocks >= target_blocks:
            return c
        best = c
    return best  # None when no tile divides rows_per_group (caller computes stats separately)


def pick_igemm3(M: int, N: int, Kc: int, taps: int, phases: int = 1, rows_per_group: Optional[int] = None,
                target_blocks: int = 2 * CU_COUNT) -> Optional[Tuple[int, int]]:
    """(cfg, splits) heuristic for igemm3: the largest 64x64-per-wave tile that fits N, then
    split-K until ~target_blocks workgroups (each split keeps >= 4 K tiles). Two LDS stages
    (21x): every layer of the in-situ tuned 128x128 step moved from 3 stages to 2
    (profiles/r3/tune_insitu_128_r3.txt), as most 64x64 entries had."""
    if N >= 128:
        order = [210, 211, 213, 215]
    elif N >= 64:
        order = [211, 213, 215]
    else:
        return None
    kt = taps * -(-Kc // 64)
    for c in order:
        bm, bn = IGEMM3_TILES[c % 10]
        if rows_per_group is not None and rows_per_group % bm != 0:
            continue
        tiles = -(-M // bm) * -(-N // bn) * phases
        sp = 1
        while tiles * sp < target_blocks and kt // (sp * 2) >= 4 and sp < 8:
            sp *= 2
        if tiles * sp >= target_blocks // 2 or c == order[-1]:
            return c, sp
    return None


_TUNED = None
TUNED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "igemm_tuned.json")


def tuned_table() -> dict:
    """Per-layer tile choices measured on MI355X by ``benchmarks/bench_kernels.py --write``
    (key ``mode,Bn,Hin,Win,Kc,Hout,Wout,N`` -> "cfg:splits" (or a bare cfg): cfg < 200 is
    igemm.hip (+100 = LDS-DMA staging), 200..239 igemm3.hip)."""
    global _TUNED
    if _TUNED is None:
        _TUNED = {}
        path = os.environ.get("DCGAN_TUNED_PATH", TUNED_PATH)  # A/B of tile tables
        if os.environ.get("DCGAN_NO_TUNED") != "1" and os.path.exists(path):
            import json
            with open(path) as f:
                for k, v in json.load(f).items():
                    c, _, sp = str(v).partition(":")
                    _TUNED[k] = (int(c), int(sp or 1))
    return _TUNED


def igemm_cfg_for(mode: int, Bn: int, Hin: int, Win: int, Kc: int, Hout: int, Wout: int, N: int,
                  rows_per_group: Optional[int] = None, bkn: bool = False,
                  dtype: int = 0) -> Optional[Tuple[int, int]]:
    """(cfg, splits) for one implicit-GEMM launch: the tuned entry when present and legal
    (weight layout, BN-statistics grouping), else the heuristics. None when no tile can
    produce group-aligned statistics (caller computes them in a separate pass). dtype 2 =
    the fp32 build (its own tile family, no tuned table)."""
    if mode == 1:
        M, phases, taps = Bn * (-(-Hout // 2)) * (-(-Wout // 2)), 4, 9
    else:
        M, phases, taps = Bn * Hout * Wout, 1, (25 if mode == 0 else 1)
    if dtype == 2:
        if mode == 1 and rows_per_group is not None:
            return None
        return pick_igemm_f32(M, N, phases, rows_per_group)
    ent = tuned_table().get("%d,%d,%d,%d,%d,%d,%d,%d" % (mode, Bn, Hin, Win, Kc, Hout, Wout, N))
    if ent is not None:
        cfg, sp = ent
        ok = (cfg >= 200 and igemm3_pp_ok(cfg, mode, Kc)) or (not bkn and sp == 1 and cfg % 100 in IGEMM_CFGS)
        if cfg >= 300:
            ok = halo_ok(cfg, mode, Bn, Hout, Wout, Kc, bkn, sp)
        if ok and (rows_per_group is None or rows_per_group % tile_of(cfg)[0] == 0):
            return cfg, sp
    if N % 8 == 0 and N >= 64:
        r = pick_igemm3(M, N, Kc, taps, phases, rows_per_group)
        if r is not None:
            return r
    if bkn:
        return None
    c = pick_igemm_cfg(M, N, phases, rows_per_group)
    return None if c is None else (c, 1)


def pick_wgrad(Mc: int, Nc: int, K: int, taps: int, target_blocks: int = 4 * CU_COUNT,
               dtype: int = 0) -> Tuple[int, int]:
    """(cfg, splits) for a weight-gradient GEMM of Mc x Nc per tap over K pixels (dtype 2:
    the fp32 kernel, one 64x64 tile for every cfg)."""
    if dtype == 2:
        tiles = -(-Mc // 64) * -(-Nc // 64) * taps
        kt = -(-K // 64)
        return 3, max(1, min(-(-target_blocks // tiles), max(1, kt // (16 if taps == 1 else 4))))
    if Mc >= 128 and Nc >= 128:
        cfg = 0
    elif Mc < 128 and Nc >= 128:
        cfg = 1 if Mc > 32 else 4
    elif Mc >= 128 and Nc < 128:
        cfg = 2 if Nc > 32 else 5
    elif Mc > 32 and Nc > 32:
        cfg = 3
    elif Nc > 32:
        cfg = 4
    elif Mc > 32:
        cfg = 5
    else:
        cfg = 6
    bm, bn = WGRAD_CFGS[cfg]
    tiles = -(-Mc // bm) * -(-Nc // bn) * taps
    kt = -(-K // 64)
    # plain (im2col'd, 1-tap) layers reduce over up to 2^18 pixels into a tiny 80 x 64 matrix:
    # >= 16 k-tiles per split keeps the slab traffic (splits x Mc x Nc fp32) and the reduce short
    min_kt = 16 if taps == 1 else 4
    splits = max(1, min(-(-target_blocks // tiles), max(1, kt // min_kt)))
    return cfg, splits


WGRAD3_TILES = {0: (128, 128), 1: (64, 128), 2: (128, 64), 3: (64, 64)}
# wgrad5.hip (csrc/hip/wgrad5.hip, cfg 400 + id): (Mc, BN, Wd, LDS stages) -- a workgroup owns one
# kernel row (5 taps) x all Mc x BN channels, a k-tile is 64 / Wd whole output rows of one image
WGRAD5_CFGS = {400: (64, 64, 16, 2), 401: (64, 64, 16, 3), 402: (64, 64, 8, 2), 403: (64, 64, 32, 2),
               404: (128, 64, 8, 2), 405: (128, 64, 16, 2), 406: (128, 32, 8, 2), 407: (128, 32, 16, 2),
               408: (64, 64, 64, 2), 409: (64, 64, 4, 2)}
# 410 + id: the same tiles with the split-K sum in a second, GPU-wide kernel (no last-arrival tail)
WGRAD5_CFGS.update({c + 10: v for c, v in list(WGRAD5_CFGS.items())})


def wgrad5_fits(cfg: int, Mc: int, Hd: int, Wd: int, Bn: int = 64) -> bool:
    """wgrad5 cfg usable for a layer: whole channel blocks, its output width, whole output rows
    per 64-pixel k-tile (a fraction of one image or whole images), whole k-tiles."""
    ent = WGRAD5_CFGS.get(cfg)
    if ent is None or Mc % ent[0] or ent[2] != Wd:
        return False
    R = 64 // Wd
    return (Hd % R == 0 or R % Hd == 0) and (Bn * Hd * Wd) % 64 == 0


def pick_wgrad3(Mc: int, Nc: int, K: int, target_blocks: int = 2 * CU_COUNT) -> Optional[Tuple[int, int]]:
    """(cfg, splits) heuristic for wgrad3.hip (25-tap gather GEMM, in-kernel split-K): the
    largest tile not wider than the operands, split-K until ~target_blocks workgroups while
    every split keeps >= 8 k-tiles of 64 pixels. None -> wgrad.hip."""
    if Mc % 8 or Nc % 8 or Mc < 64 or Nc < 64:
        return None
    kt = -(-K // 64)
    for tid in (0, 1, 2, 3):
        bm, bn = WGRAD3_TILES[tid]
        if bm > Mc or bn > Nc:
            continue
        tiles = -(-Mc // bm) * -(-Nc // bn) * 25
        sp = 1
        while tiles * sp < target_blocks and kt // (2 * sp) >= 8 and sp < 16:
            sp *= 2
        return 310 + tid, sp  # two LDS stages (31x), as every tuned 64x64 entry
    return None


def wgrad3_key(Mc: int, Nc: int, Bn: int, Hd: int, Wd: int, Hg: int) -> str:
    return "w3,%d,%d,%d,%d,%d,%d" % (Mc, Nc, Bn, Hd, Wd, Hg)


def wgrad_splits_for(Mc: int, Nc: int, Bn: int, Hd: int, Wd: int, Hg: int) -> Optional[int]:
    """Tuned split count for wgrad.hip on a 25-tap layer (entry "0:splits"), or None."""
    ent = tuned_table().get(wgrad3_key(Mc, Nc, Bn, Hd, Wd, Hg))
    return ent[1] if ent is not None and ent[0] == 0 and ent[1] >= 1 else None


def wgrad3_cfg_for(Mc: int, Nc: int, Bn: int, Hd: int, Wd: int, Hg: int) -> Optional[Tuple[int, int]]:
    """(cfg, splits) for a 25-tap weight gradient on wgrad3.hip, or None to keep wgrad.hip:
    the tuned entry (benchmarks/bench_wgrad.py --write; cfg 0 = wgrad.hip measured faster),
    else the heuristic."""
    if os.environ.get("DCGAN_NO_WGRAD3") == "1":
        return None
    ent = tuned_table().get(wgrad3_key(Mc, Nc, Bn, Hd, Wd, Hg))
    if ent is not None:
        return None if ent[0] == 0 else ent
    return pick_wgrad3(Mc, Nc, Bn * Hd * Wd)


# --------------------------------------------------------------------------- one-shot wrappers
def _check_bf16(*ts):
    for t in ts:
        if t is not None and (t.dtype not in (torch.bfloat16, torch.float16) or not t.is_contiguous()
                              or not t.is_cuda):
            raise ValueError("expected contiguous cuda bf16 tensor, got %s %s" % (t.dtype, t.device))


def pack_conv_weight(w: torch.Tensor, kind: str, use: str) -> torch.Tensor:
    """bf16 B-operand layout [25][N][Kc] for the igemm kernel.

    conv weight HWIO [5,5,ci,co]: use='fwd' -> [25][co][ci] (transposed), 'dgrad' -> natural.
    deconv weight [5,5,co,ci]:    use='fwd' -> natural,              'dgrad' -> [25][ci][co]."""
    w = w.reshape(25, w.shape[2], w.shape[3])
    transpose = (kind == "conv" and use == "fwd") or (kind == "deconv" and use == "dgrad")
    if transpose:
        w = w.transpose(1, 2)
    return w.contiguous().to(torch.bfloat16)


def pack_im2col_weight(w: torch.Tensor, kind: str, kpad: int) -> torch.Tensor:
    """[N][kpad] bf16 for a 3-channel layer run as a plain GEMM over im2col rows.
    conv (D L0) HWIO [5,5,3,co] -> Bt[co][tap*3+ci]; deconv dgrad (G last) [5,5,3,ci]:
    Bt[ci][tap*3+co]."""
    A = w.shape[2]
    t = w.reshape(25 * A, w.shape[3]).t()  # [N][25*A], k = tap*A + a
    out = torch.zeros(t.shape[0], kpad, dtype=torch.bfloat16, device=w.device)
    out[:, :25 * A] = t.to(torch.bfloat16)
    return out


def conv2d_same(x: torch.Tensor, w_packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor] = None,
                act: Optional[str] = None, leak: float = 0.2, stats: bool = False, out_f32: bool = False,
                cfg: Optional[int] = None, bkn: bool = False, splits: int = 1):
    """TF-SAME stride-2 5x5 conv on the HIP igemm kernel. x bf16 NHWC [B,H,W,Ci] (Ci % 8 == 0),
    w_packed bf16 [25][co][ci] (bkn=True: [25][ci][co], i.e. the HWIO weight itself; cfg >= 200).
    Returns y (and per-tile stats partials [P,2,co] if stats)."""
    _check_bf16(x, w_packed)
    B, H, W, Ci = x.shape
    Ho, Wo = same_out(H), same_out(W)
    py, px = same_pads(H)[0], same_pads(W)[0]
    M = B * Ho * Wo
    cfg = pick_igemm_cfg(M, cout) if cfg is None else cfg
    bm, bn = tile_of(cfg)
    y = torch.empty(B, Ho, Wo, cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    mt = -(-M // bm)
    st = torch.empty(mt, 2, cout, device=x.device, dtype=torch.float32) if stats else None
    prog = ext().Program()
    prog.igemm_ex("conv", 0, _p(x), _p(w_packed), _p(y), B, H, W, Ci, Ho, Wo, cout, py, px, cfg, int(out_f32), cout,
                  0, _p(bias), ACT[act], leak, _p(st), 0, int(bkn), -1, splits)
    run(prog)
    return (y, st) if stats else y


def conv2d_transpose_same(x: torch.Tensor, w_packed: torch.Tensor, cout: int, out_hw: Tuple[int, int],
                          bias: Optional[torch.Tensor] = None, act: Optional[str] = None, leak: float = 0.2,
                          stats: bool = False, out_f32: bool = False, cfg: Optional[int] = None,
                          bkn: bool = False, splits: int = 1):
    """TF-SAME stride-2 5x5 conv_transpose via 4 sub-pixel phases. x bf16 [B,Hi,Wi,Ci],
    w_packed bf16 [25][co][ci] (bkn=True: [25][ci][co]; cfg >= 200)."""
    _check_bf16(x, w_packed)
    B, Hi, Wi, Ci = x.shape
    Ho, Wo = out_hw
    py, px = same_pads(Ho)[0], same_pads(Wo)[0]
    Mphase = B * (-(-Ho // 2)) * (-(-Wo // 2))
    cfg = pick_igemm_cfg(Mphase, cout, phases=4) if cfg is None else cfg
    bm, bn = tile_of(cfg)
    y = torch.empty(B, Ho, Wo, cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    prog = ext().Program()
    st = None
    if stats:
        mt = -(-Mphase // bm)
        st = torch.empty(mt * 4, 2, cout, device=x.device, dtype=torch.float32)
    prog.igemm_ex("deconv", 1, _p(x), _p(w_packed), _p(y), B, Hi, Wi, Ci, Ho, Wo, cout, py, px, cfg, int(out_f32),
                  cout, 0, _p(bias), ACT[act], leak, _p(st), 0, int(bkn), -1, splits)
    run(prog)
    return (y, st) if stats else y


NCONV_MAX_GRID = 512  # persistent workgroups of nconv (2 per CU: the kernel's occupancy)


def nconv_grid(prog, B: int, Ho: int, Wo: int, cap: Optional[int] = None) -> int:
    """Workgroup count of an nconv launch (= its BN-backward partial rows): persistent (cap
    workgroups looping over the tiles) or, with cap <= 0, one workgroup per tile. The default cap
    is NCONV_MAX_GRID; DCGAN_NCONV_CAP overrides it (A/B studies)."""
    if cap is None:
        v = os.environ.get("DCGAN_NCONV_CAP", str(NCONV_MAX_GRID))
        if not v.isdigit():
            raise ValueError("DCGAN_NCONV_CAP must be a non-negative integer (0 = one workgroup per tile), "
                             "got %r" % v)
        cap = int(v)
    tiles = prog.nconv_tiles(B, Ho, Wo)
    return tiles if cap <= 0 else min(tiles, cap)


def nconv(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
          leak: float = 0.2, bnb: Optional[tuple] = None):
    """TF-SAME stride-2 5x5 conv with Cin <= 4 and Cout = 64 on narrow2.hip's persistent MFMA
    kernel. x [B,H,W,Cin], w HWIO [5,5,Cin,64]. bnb = (bx, by, mean[64], rstd[64], act): also
    the BN-backward partial statistics (sum g, sum g*xhat), g = y_out * act'(by) -- returned as
    [grid][2][64] next to the output."""
    _check_bf16(x, w)
    B, Hh, Ww, C = x.shape
    Ho, Wo = -(-Hh // 2), -(-Ww // 2)
    y = torch.empty(B, Ho, Wo, 64, device=x.device, dtype=x.dtype)
    prog = ext().Program(x.dtype == torch.float16)
    grid = nconv_grid(prog, B, Ho, Wo)
    part = torch.empty(grid, 2, 64, device=x.device) if bnb is not None else None
    bx, by, mean, rstd, bact = bnb if bnb is not None else (None, None, None, None, None)
    prog.nconv("nconv", _p(x), _p(w), _p(bias), _p(y), B, Hh, Ww, C, Ho, Wo, same_pads(Hh)[0], same_pads(Ww)[0],
               ACT[act], leak, grid, _p(bx), _p(by), _p(mean), _p(rstd), ACT[bact], leak, _p(part), 0)
    run(prog)
    return (y, part) if bnb is not None else y


def nwgrad(x: torch.Tensor, d: torch.Tensor, pad: int) -> torch.Tensor:
    """Weight gradient of a 1..4-channel stride-2 5x5 layer (narrow2.hip): out[25][Cin][64] =
    sum over d's pixels of the stride-2 window of x (top/left padding `pad`) times d."""
    _check_bf16(x, d)
    B, Hh, Ww, C = x.shape
    _, Hd, Wd, N = d.shape
    assert N == 64
    out = torch.empty(25, C, 64, device=x.device)
    prog = ext().Program(x.dtype == torch.float16)
    prog.nwgrad("nwgrad", _p(x), B, Hh, Ww, C, _p(d), Hd, Wd, pad, _p(out), 0)
    run(prog)
    return out


def narrow_deconv(x: torch.Tensor, w: torch.Tensor, out_hw: Tuple[int, int], bias: Optional[torch.Tensor] = None,
                  act: Optional[str] = None, leak: float = 0.2) -> torch.Tensor:
    """TF-SAME stride-2 5x5 conv_transpose with N <= 4 output channels on the direct VALU
    kernel. x [B,Hi,Wi,C] (C % 8 == 0), w [25][N][C] (the TF deconv layout [5,5,N,C], or a
    conv's HWIO [5,5,N=ci,C=co] for its data gradient)."""
    _check_bf16(x, w)
    B, Hi, Wi, C = x.shape
    N = w.numel() // (25 * C)
    Ho, Wo = out_hw
    y = torch.empty(B, Ho, Wo, N, device=x.device, dtype=x.dtype)
    prog = ext().Program(x.dtype == torch.float16)
    prog.narrow_deconv("narrow", _p(x), _p(w), _p(bias), _p(y), B, Hi, Wi, C, Ho, Wo, N, same_pads(Ho)[0],
                       ACT[act], leak, 0)
    run(prog)
    return y


def gemm_plain(a: torch.Tensor, bt: torch.Tensor, out_f32: bool = False, bias=None, act=None,
               cfg: Optional[int] = None, bkn: bool = False, splits: int = 1) -> torch.Tensor:
    """C[M][N] = A[M][K] . Bt[N][K] (bf16, K % 8 == 0). bkn=True: bt is B[Kb][N] (n contiguous,
    Kb <= K rows; rows Kb..K-1 read as zeros -- the im2col K padding)."""
    _check_bf16(a, bt)
    M, K = a.shape
    N = bt.shape[1] if bkn else bt.shape[0]
    kb = bt.shape[0] if bkn else -1
    cfg = pick_igemm_cfg(M, N) if cfg is None else cfg
    c = torch.empty(M, N, device=a.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    prog = ext().Program()
    prog.igemm_ex("gemm", 2, _p(a), _p(bt), _p(c), M, 1, 1, K, 1, 1, N, 0, 0, cfg, int(out_f32), N, 0, _p(bias),
                  ACT[act], 0.2, 0, 0, int(bkn), kb, splits)
    run(prog)
    return c


def conv_wgrad(g_src: torch.Tensor, dm: torch.Tensor, pad: int, mode: int = 0, cfg=None, splits=None) -> torch.Tensor:
    """out[25][Mc][Nc] = sum_k G[b,2y+ky-pad,2x+kx-pad,m] * Dm[b,y,x,n] (fp32).
    mode 2: g_src is an im2col matrix [K][Mc] and the result is [Mc][Nc]."""
    _check_bf16(g_src, dm)
    if mode == 2:
        K, Mc = g_src.shape
        Nc = dm.shape[-1]
        Bn, Hd, Wd = K, 1, 1
        Hg = Wg = 1
        taps = 1
    else:
        Bn, Hg, Wg, Mc = g_src.shape
        _, Hd, Wd, Nc = dm.shape
        taps = 25
        K = Bn * Hd * Wd
    c, s = pick_wgrad(Mc, Nc, K, taps)
    cfg = c if cfg is None else cfg
    splits = s if splits is None else splits
    slabs = torch.empty(splits, taps, Mc, Nc, device=dm.device, dtype=torch.float32)
    out = torch.empty(taps, Mc, Nc, device=dm.device, dtype=torch.float32)
    prog = ext().Program()
    prog.wgrad("wgrad", mode, _p(g_src), Hg, Wg, Mc, _p(dm), Bn, Hd, Wd, Nc, pad, cfg, splits, _p(slabs), _p(out),
               out.numel(), 1.0, 0)
    run(prog)
    return out if mode != 2 else out[0]


def conv_wgrad3(g_src: torch.Tensor, dm: torch.Tensor, pad: int, cfg: Optional[int] = None,
                splits: Optional[int] = None, scale: float = 1.0) -> torch.Tensor:
    """wgrad3.hip: out[25][Mc][Nc] = scale * sum_k G[b,2y+ky-pad,2x+kx-pad,m] * Dm[b,y,x,n] (fp32)."""
    _check_bf16(g_src, dm)
    Bn, Hg, Wg, Mc = g_src.shape
    _, Hd, Wd, Nc = dm.shape
    if cfg is None or splits is None:
        plan = pick_wgrad3(Mc, Nc, Bn * Hd * Wd)
        if plan is None:
            raise ValueError("no wgrad3 tile for Mc=%d Nc=%d" % (Mc, Nc))
        cfg = plan[0] if cfg is None else cfg
        splits = plan[1] if splits is None else splits
    out = torch.empty(25, Mc, Nc, device=dm.device, dtype=torch.float32)
    prog = ext().Program(g_src.dtype == torch.float16)
    prog.wgrad3("wgrad3", _p(g_src), Hg, Wg, Mc, _p(dm), Bn, Hd, Wd, Nc, pad, cfg, splits, _p(out), scale, 0)
    run(prog)
    return out


def act_bwd_dbias(dy: torch.Tensor, y: torch.Tensor, act: int, leak: float = 0.2):
    """(dx, db): dx = dy * act'(y) (elem dtype), db[c] = sum over rows of dx (fp32) -- one launch."""
    _check_bf16(dy, y)
    C = dy.shape[-1]
    R = dy.numel() // C
    dx = torch.empty_like(dy)
    db = torch.empty(C, device=dy.device, dtype=torch.float32)
    prog = ext().Program(dy.dtype == torch.float16)
    prog.act_bwd_dbias("abd", _p(dy), _p(y), _p(dx), R, C, act, leak, _p(db), 0)
    run(prog)
    return dx, db


def head_bwd(x: torch.Tensor, dl: torch.Tensor, w: torch.Tensor):
    """(dx, dW, db) of logits = x @ w + b: dW = x^T dl, db = sum dl, dx = dl w^T (elem dtype)."""
    _check_bf16(x)
    R, K = x.shape
    dx = torch.empty_like(x)
    dW = torch.empty(K, device=x.device, dtype=torch.float32)
    db = torch.empty(1, device=x.device, dtype=torch.float32)
    prog = ext().Program(x.dtype == torch.float16)
    prog.head_bwd("hb", _p(x), _p(dl), _p(w), _p(dx), _p(dW), _p(db), R, K, 0)
    run(prog)
    return dx, dW, db


def im2col_s2(x: torch.Tensor, kpad: int) -> torch.Tensor:
    _check_bf16(x)
    B, H, W, C = x.shape
    Ho, Wo = same_out(H), same_out(W)
    out = torch.empty(B * Ho * Wo, kpad, device=x.device, dtype=torch.bfloat16)
    prog = ext().Program()
    prog.im2col_s2("im2col", _p(x), _p(out), B, H, W, C, Ho, Wo, same_pads(H)[0], same_pads(W)[0], kpad, 0)
    run(prog)
    return out


def adam_(w: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, powers: torch.Tensor, lr: float,
          beta1: float, beta2: float, eps: float, gscale: float = 1.0, advance_powers: bool = True) -> None:
    prog = ext().Program()
    prog.adam("adam", _p(w), _p(g), _p(m), _p(v), _p(powers), w.numel(), lr, beta1, beta2, eps, gscale, 0)
    if advance_powers:
        prog.step_end("powers", _p(powers), 0, beta1, beta2, 0.0, 0.0, 0, 0)
    run(prog)

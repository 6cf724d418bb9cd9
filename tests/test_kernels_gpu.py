"""Single-kernel parity on the GPU: MFMA dense layer, implicit-GEMM 3x3 conv forward / transposed conv,
and the device RNG — each against a plain fp32 reference of the same op (torch CPU / numpy)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import rng

pytestmark = pytest.mark.gpu


def _lib():
    from vad_amd import _native
    return _native


@pytest.mark.parametrize("M,K,N,relu", [(128, 6144, 512, 1), (8, 6144, 512, 1), (37, 64, 20, 0), (5, 64, 2, 0),
                                        (256, 96, 130, 1)])
def test_dense_forward(M, K, N, relu):
    nat = _lib()
    g = torch.Generator().manual_seed(M * 1000 + N)
    X = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    ref = X @ W.T + b
    if relu:
        ref = ref.clamp_min(0)
    d = torch.device("cuda")
    Y = torch.empty(M, N, device=d)
    scratch = torch.empty(1 << 22, device=d)
    Xd, Wd, bd = X.to(d), W.to(d), b.to(d)  # keep the device copies alive until the kernel ran
    nat.check(nat.lib().vad_dense_forward(Xd.data_ptr(), M, K, Wd.data_ptr(), bd.data_ptr(), N,
                                          Y.data_ptr(), relu, scratch.data_ptr(), scratch.numel(),
                                          nat.stream_of(d)))
    torch.cuda.synchronize()
    np.testing.assert_allclose(Y.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


CONV_CASES = [(2, 32, 32, 19, 17, 1), (2, 32, 64, 29, 29, 2), (1, 64, 128, 15, 15, 2), (2, 128, 256, 8, 8, 1),
              (3, 64, 64, 10, 7, 2), (1, 256, 256, 8, 8, 1),
              # stride-1 shapes of the LDS-patch kernels: 2x8x8 tiles with odd NF, 8x16, 4x32 (57-wide, ragged)
              (3, 32, 32, 8, 8, 1), (2, 64, 64, 15, 15, 1), (1, 32, 32, 57, 57, 1), (2, 128, 128, 29, 29, 1),
              (2, 32, 64, 5, 3, 1),
              # stride-2 patch geometries (4x32 / 8x16 / 2x8x8 forward tiles, 16x16 dX parity tiles), odd sizes
              (2, 32, 64, 57, 57, 2), (3, 128, 256, 16, 16, 2), (1, 64, 128, 31, 18, 2)]


def _conv_path(nat, patch):
    nat.lib().vad_set_tuning(b"conv_patch", 1 if patch else 0)
    nat.lib().vad_set_tuning(b"conv_patch_persist", 0 if patch == 2 else 1)
    nat.lib().vad_set_tuning(b"conv_split", 1 if patch == 3 else 0)


def _conv_default(nat):
    nat.lib().vad_set_tuning(b"conv_patch", 1)
    nat.lib().vad_set_tuning(b"conv_patch_persist", 1)
    nat.lib().vad_set_tuning(b"conv_split", 1)


@pytest.mark.parametrize("patch", [3, 1, 0, 2])
@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", CONV_CASES)
def test_conv3x3_forward_and_dgrad(NF, Ci, Co, IH, IW, s, patch):
    """patch 3: split-bf16 patch kernels (conv_x3.hip; stride-2 input gradients on the split parity-class kernel),
    1: f32 LDS-patch kernels (persistent variant for 32-channel stride-1 layers), 2: f32 patch kernels without the
    persistent variant, 0: implicit-GEMM path."""
    nat = _lib()
    _conv_path(nat, patch)
    g = torch.Generator().manual_seed(NF * 7 + Ci + Co + IH)
    x = torch.randn(NF, Ci, IH, IW, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
    bias = torch.randn(Co, generator=g)
    ref = F.conv2d(x, w, bias, stride=s, padding=1)
    OH, OW = ref.shape[2:]
    d = torch.device("cuda")
    xh = x.permute(0, 2, 3, 1).contiguous().to(d)
    y = torch.empty(NF, OH, OW, Co, device=d)
    wf = torch.empty(9 * Ci * Co, device=d)
    wd = torch.empty(9 * Ci * Co, device=d)
    parts = torch.empty((NF * OH * OW // 64 + 2) * 2 * Co, device=d)
    wdev = w.contiguous().to(d)
    st = nat.stream_of(d)
    bd = bias.to(d)
    nat.check(nat.lib().vad_conv3x3_forward(xh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), bd.data_ptr(),
                                            Co, s, y.data_ptr(), wf.data_ptr(), wd.data_ptr(), parts.data_ptr(), st))
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().permute(0, 3, 1, 2).numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    # transposed conv (input gradient)
    dy = torch.randn(NF, Co, OH, OW, generator=g)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, bias, stride=s, padding=1).backward(dy)
    dx = torch.empty(NF, IH, IW, Ci, device=d)
    dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
    nat.check(nat.lib().vad_conv3x3_dgrad(dyh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), Co, s, dx.data_ptr(),
                                          wf.data_ptr(), wd.data_ptr(), st))
    torch.cuda.synchronize()
    _conv_default(nat)
    np.testing.assert_allclose(dx.cpu().permute(0, 3, 1, 2).numpy(), xr.grad.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", [(2, 64, 64, 29, 29, 1), (2, 32, 64, 57, 57, 2), (1, 256, 256, 8, 8, 1)])
def test_conv3x3_split_accuracy_matches_f32(NF, Ci, Co, IH, IW, s):
    """The split-bf16 kernels (three bf16 planes per fp32 operand, six products per K step) against an fp64
    reference: their worst error, relative to sum |x||w| of each output, is within 2x that of the exact-f32 MFMA
    patch kernels (both are ~1e-7; a plain bf16 conv would sit near 4e-3)."""
    nat = _lib()
    g = torch.Generator().manual_seed(5 + Ci + IH)
    x = torch.randn(NF, Ci, IH, IW, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
    bias = torch.zeros(Co)
    ref = F.conv2d(x.double(), w.double(), bias.double(), stride=s, padding=1)
    mag = F.conv2d(x.double().abs(), w.double().abs(), None, stride=s, padding=1)
    OH, OW = ref.shape[2:]
    d = torch.device("cuda")
    xh = x.permute(0, 2, 3, 1).contiguous().to(d)
    wdev, bd = w.contiguous().to(d), bias.to(d)
    errs = {}
    for patch in (1, 3):
        _conv_path(nat, patch)
        y = torch.empty(NF, OH, OW, Co, device=d)
        wf = torch.empty(9 * Ci * Co, device=d)
        wd = torch.empty(9 * Ci * Co, device=d)
        parts = torch.empty((NF * OH * OW // 64 + 2) * 2 * Co, device=d)
        nat.check(nat.lib().vad_conv3x3_forward(xh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), bd.data_ptr(), Co, s,
                                                y.data_ptr(), wf.data_ptr(), wd.data_ptr(), parts.data_ptr(),
                                                nat.stream_of(d)))
        torch.cuda.synchronize()
        out = y.cpu().permute(0, 3, 1, 2).double()
        errs[patch] = float(((out - ref).abs() / mag).max())
    _conv_default(nat)
    assert errs[3] < 1e-6, errs
    assert errs[3] <= 2.0 * errs[1] + 1e-8, errs


@pytest.mark.parametrize("NF,Ci,Co,IH,IW", [(2, 32, 64, 57, 57), (3, 64, 128, 29, 29), (4, 128, 256, 15, 15),
                                            (2, 64, 128, 31, 18)])
def test_conv3x3_dgrad_s2_split_accuracy_matches_f32(NF, Ci, Co, IH, IW):
    """Stride-2 input gradient on the split-bf16 parity-class kernel against an fp64 reference: worst error relative
    to sum |dy||w| within 2x that of the exact-f32 parity kernel (both ~1e-7)."""
    nat = _lib()
    g = torch.Generator().manual_seed(17 + Ci + IH)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
    OH, OW = (IH - 1) // 2 + 1, (IW - 1) // 2 + 1
    dy = torch.randn(NF, Co, OH, OW, generator=g)
    ref = torch.nn.grad.conv2d_input((NF, Ci, IH, IW), w.double(), dy.double(), stride=2, padding=1)
    mag = torch.nn.grad.conv2d_input((NF, Ci, IH, IW), w.double().abs(), dy.double().abs(), stride=2, padding=1)
    d = torch.device("cuda")
    dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
    wdev = w.contiguous().to(d)
    wf = torch.empty(9 * Ci * Co, device=d)
    wd = torch.empty(9 * Ci * Co, device=d)
    errs = {}
    for split in (0, 1):
        nat.lib().vad_set_tuning(b"conv_dgrad_s2_x3", split)
        dx = torch.empty(NF, IH, IW, Ci, device=d)
        nat.check(nat.lib().vad_conv3x3_dgrad(dyh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), Co, 2, dx.data_ptr(),
                                              wf.data_ptr(), wd.data_ptr(), nat.stream_of(d)))
        torch.cuda.synchronize()
        errs[split] = float(((dx.cpu().permute(0, 3, 1, 2).double() - ref).abs() / (mag + 1e-30)).max())
    nat.lib().vad_set_tuning(b"conv_dgrad_s2_x3", 1)
    assert errs[1] < 1e-6, errs
    assert errs[1] <= 2.0 * errs[0] + 1e-8, errs


@pytest.mark.parametrize("stream", [rng.S_DET_DROP1, rng.S_EPS, rng.S_INPUT])
def test_device_rng_bitexact(stream):
    nat = _lib()
    d = torch.device("cuda")
    out = torch.empty(37, 300, dtype=torch.int32, device=d)
    nat.check(nat.lib().vad_rng_u24(12345, stream, 7, 1000, 37, 300, out.data_ptr(), nat.stream_of(d)))
    ref = rng.u24(12345, stream, 7, np.arange(1000, 1037), np.arange(300))
    np.testing.assert_array_equal(out.cpu().numpy().astype(np.int64), ref)


def test_device_synth_frames_bitexact():
    nat = _lib()
    d = torch.device("cuda")
    out = torch.empty(6, 51 * 40, device=d)
    nat.check(nat.lib().vad_synth_frames(3, 1, 10, 6, 51 * 40, 0, out.data_ptr(), nat.stream_of(d)))
    u8 = rng.pixels_u8(3, 1, 10, 6, 51 * 40).astype(np.float32)
    np.testing.assert_array_equal(out.cpu().numpy(), (u8 - np.float32(0.5)) / np.float32(0.5))


WGRAD_CASES = [(2, 32, 32, 19, 17, 1), (32, 256, 256, 8, 8, 1), (32, 128, 256, 15, 15, 2), (32, 32, 32, 57, 57, 1),
               (8, 64, 64, 29, 29, 1), (3, 64, 128, 15, 15, 2),
               # LDS-patch geometries: stride-2 4x32 tiles, 2x8x8 tiles with odd NF (both strides), tiny frames
               (3, 32, 64, 57, 57, 2), (5, 64, 64, 8, 8, 1), (3, 128, 256, 15, 15, 2), (2, 32, 32, 5, 3, 1),
               # stride-2 split-bf16 geometries: 4x16 tiles with a ragged width, frames smaller than a tile
               (3, 64, 128, 29, 30, 2), (2, 32, 32, 5, 3, 2),
               # stride-1 multi-co-tile geometries (4x16 and 8x8 tiles, 64 co per block)
               (3, 128, 128, 15, 15, 1), (2, 64, 64, 13, 11, 1),
               # 32-output-channel stride-2 layers on the transposed-read kernel (8x8 and 4x16 tiles, one co tile)
               (2, 32, 32, 15, 15, 2), (3, 32, 32, 33, 31, 2), (2, 64, 32, 9, 40, 2)]


def _wgrad_path(nat, patch):
    """3: split-bf16 transposed-read kernel for both strides (default, conv_x3w.hip), 4: the
    older split-bf16 kernels (conv_x3.hip), 1: f32 LDS-patch kernel for stride-1 layers, 2: f32 LDS-patch kernel for all strides, 0:
    implicit-GEMM path."""
    split = patch in (3, 4)
    nat.lib().vad_set_tuning(b"conv_wgrad_patch", 1 if split else patch)
    nat.lib().vad_set_tuning(b"conv_wgrad_split", 1 if split else 0)
    nat.lib().vad_set_tuning(b"conv_wgrad_split_s2", 1 if split else 0)
    nat.lib().vad_set_tuning(b"conv_wgrad_tr", 1 if patch == 3 else 0)


@pytest.mark.parametrize("patch", [3, 4, 1, 0, 2])
@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", WGRAD_CASES)
def test_conv3x3_wgrad(NF, Ci, Co, IH, IW, s, patch):
    nat = _lib()
    _wgrad_path(nat, patch)
    g = torch.Generator().manual_seed(NF * 5 + Ci + Co + IH)
    x = torch.randn(NF, Ci, IH, IW, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, stride=s, padding=1)
    dy = torch.randn_like(y)
    y.backward(dy)
    d = torch.device("cuda")
    xh = x.permute(0, 2, 3, 1).contiguous().to(d)
    dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
    dW = torch.empty(Co, Ci, 3, 3, device=d)
    part = torch.empty(1 << 24, device=d)
    nat.check(nat.lib().vad_conv3x3_wgrad(xh.data_ptr(), dyh.data_ptr(), NF, Ci, IH, IW, Co, s, dW.data_ptr(),
                                          part.data_ptr(), part.numel(), nat.stream_of(d)))
    torch.cuda.synchronize()
    _wgrad_path(nat, 3)
    ref = wr.grad
    np.testing.assert_allclose(dW.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4 * float(ref.abs().max()))


@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", [(8, 32, 32, 57, 57, 1), (4, 64, 64, 29, 29, 1), (16, 256, 256, 8, 8, 1),
                                              (6, 128, 128, 15, 15, 1),
                                              # the backbone's stride-2 layers (2x32, 4x16, 8x8 tiles)
                                              (8, 32, 64, 57, 57, 2), (6, 64, 128, 29, 29, 2),
                                              (8, 128, 256, 15, 15, 2)])
def test_conv3x3_wgrad_split_accuracy_matches_f32(NF, Ci, Co, IH, IW, s):
    """Split-bf16 weight gradients (transposed-read kernel 3, older kernels 4) against an fp64 reference: worst error
    relative to sum_p |dy||x| of each weight within 2x that of the exact-f32 MFMA kernel (a plain bf16 product would
    sit near 4e-3)."""
    nat = _lib()
    g = torch.Generator().manual_seed(11 + Ci + IH + s)
    x = torch.randn(NF, Ci, IH, IW, generator=g)
    OH, OW = (IH - 1) // s + 1, (IW - 1) // s + 1
    dy = torch.randn(NF, Co, OH, OW, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (Co, Ci, 3, 3), dy.double(), stride=s, padding=1)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), (Co, Ci, 3, 3), dy.double().abs(), stride=s, padding=1)
    d = torch.device("cuda")
    xh = x.permute(0, 2, 3, 1).contiguous().to(d)
    dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
    part = torch.empty(1 << 24, device=d)
    errs = {}
    for patch in ((1, 3, 4) if s == 1 else (2, 3, 4)):
        _wgrad_path(nat, patch)
        dW = torch.empty(Co, Ci, 3, 3, device=d)
        nat.check(nat.lib().vad_conv3x3_wgrad(xh.data_ptr(), dyh.data_ptr(), NF, Ci, IH, IW, Co, s, dW.data_ptr(),
                                              part.data_ptr(), part.numel(), nat.stream_of(d)))
        torch.cuda.synchronize()
        errs[patch] = float(((dW.cpu().double() - ref).abs() / mag).max())
    _wgrad_path(nat, 3)
    for k in (3, 4):
        assert errs[k] < 1e-6, errs
        assert errs[k] <= 2.0 * errs[1 if s == 1 else 2] + 1e-8, errs


def _bf16(t):
    return t.bfloat16().double()


@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", [(2, 64, 64, 29, 29, 1), (2, 32, 64, 57, 57, 2), (3, 128, 128, 15, 15, 1),
                                              (2, 256, 256, 8, 8, 1), (2, 128, 256, 15, 15, 2)])
def test_conv3x3_bf16_mode_matches_rounded_fp64(NF, Ci, Co, IH, IW, s):
    """conv_bf16 (BASELINE config 4): operands rounded to bf16, products exact, fp32 accumulation.  Against an fp64
    conv of the bf16-rounded operands the error stays at fp32 accumulation level (< 1e-5 of sum |a||b|); stride-1
    input and weight gradients take the same path (stride-2 input gradients on the bf16 parity-class kernel)."""
    nat = _lib()
    nat.lib().vad_set_tuning(b"conv_bf16", 1)
    try:
        g = torch.Generator().manual_seed(3 + Ci + IH)
        x = torch.randn(NF, Ci, IH, IW, generator=g)
        w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
        bias = torch.zeros(Co)
        ref = F.conv2d(_bf16(x), _bf16(w), None, stride=s, padding=1)
        mag = F.conv2d(_bf16(x).abs(), _bf16(w).abs(), None, stride=s, padding=1)
        OH, OW = ref.shape[2:]
        d = torch.device("cuda")
        xh = x.permute(0, 2, 3, 1).contiguous().to(d)
        wdev, bd = w.contiguous().to(d), bias.to(d)
        y = torch.empty(NF, OH, OW, Co, device=d)
        wf = torch.empty(9 * Ci * Co, device=d)
        wd = torch.empty(9 * Ci * Co, device=d)
        parts = torch.empty((NF * OH * OW // 64 + 2) * 2 * Co, device=d)
        st = nat.stream_of(d)
        nat.check(nat.lib().vad_conv3x3_forward(xh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), bd.data_ptr(), Co, s,
                                                y.data_ptr(), wf.data_ptr(), wd.data_ptr(), parts.data_ptr(), st))
        torch.cuda.synchronize()
        err = float(((y.cpu().permute(0, 3, 1, 2).double() - ref).abs() / (mag + 1e-30)).max())
        assert err < 1e-5, err
        # the result differs from the fp32 conv by bf16 rounding, not more
        assert float((y.cpu().permute(0, 3, 1, 2) - F.conv2d(x, w, None, stride=s, padding=1)).abs().max()) < 5e-2
        dy = torch.randn(NF, Co, OH, OW, generator=g)
        dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
        dW = torch.empty(Co, Ci, 3, 3, device=d)
        part = torch.empty(1 << 24, device=d)
        nat.check(nat.lib().vad_conv3x3_wgrad(xh.data_ptr(), dyh.data_ptr(), NF, Ci, IH, IW, Co, s, dW.data_ptr(),
                                              part.data_ptr(), part.numel(), st))
        torch.cuda.synchronize()
        rdw = torch.nn.grad.conv2d_weight(_bf16(x), w.shape, _bf16(dy), stride=s, padding=1)
        mdw = torch.nn.grad.conv2d_weight(_bf16(x).abs(), w.shape, _bf16(dy).abs(), stride=s, padding=1)
        assert float(((dW.cpu().double() - rdw).abs() / (mdw + 1e-30)).max()) < 1e-5
        dx = torch.empty(NF, IH, IW, Ci, device=d)
        nat.check(nat.lib().vad_conv3x3_dgrad(dyh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), Co, s, dx.data_ptr(),
                                              wf.data_ptr(), wd.data_ptr(), st))
        torch.cuda.synchronize()
        rdx = torch.nn.grad.conv2d_input(x.shape, _bf16(w), _bf16(dy), stride=s, padding=1)
        mdx = torch.nn.grad.conv2d_input(x.shape, _bf16(w).abs(), _bf16(dy).abs(), stride=s, padding=1)
        assert float(((dx.cpu().permute(0, 3, 1, 2).double() - rdx).abs() / (mdx + 1e-30)).max()) < 1e-5
    finally:
        nat.lib().vad_set_tuning(b"conv_bf16", 0)


# native bf16 kernels (conv_bf.hip: bf16 operands AND bf16 activation storage, BASELINE config 4) -- forward of both
# strides and the stride-1 input gradient; the stride-2 input gradient and the weight gradient of that mode run the
# split kernels' bf16 instantiations.  Shapes: the config-4 layer geometries (64/32/16/8-wide maps, every channel
# pair of the backbone) plus ragged frames smaller than and straddling a tile.
BF_NATIVE_CASES = [(2, 32, 32, 64, 64, 1), (2, 32, 64, 64, 64, 2), (2, 64, 64, 32, 32, 1), (2, 64, 128, 32, 32, 2),
                   (2, 128, 128, 16, 16, 1), (3, 128, 256, 16, 16, 2), (5, 256, 256, 8, 8, 1),
                   (3, 32, 32, 19, 17, 1), (2, 64, 64, 29, 29, 1), (3, 32, 64, 57, 57, 2), (2, 128, 256, 15, 15, 2),
                   (3, 256, 256, 7, 5, 1), (1, 32, 32, 10, 7, 1), (2, 64, 128, 11, 9, 2)]


@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", BF_NATIVE_CASES)
def test_conv3x3_bf16_native_matches_rounded_fp64(NF, Ci, Co, IH, IW, s):
    """Against an fp64 conv of the bf16-rounded operands: the forward and the input gradient are fp32 accumulations
    rounded once to bf16 on store (|err| <= 2^-8 |ref| + 1e-5 sum|a||b|); the weight gradient (fp32 out) stays at
    fp32 accumulation level (1e-5 of sum |a||b|)."""
    nat = _lib()
    lib = nat.lib()
    lib.vad_set_tuning(b"conv_bf16", 1)
    lib.vad_set_tuning(b"act_bf16", 1)
    try:
        g = torch.Generator().manual_seed(11 + Ci + IH + s)
        x = torch.randn(NF, Ci, IH, IW, generator=g).bfloat16()
        w = torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5
        bias = torch.randn(Co, generator=g) * 0.1
        xd, wb = x.double(), _bf16(w)
        ref = F.conv2d(xd, wb, bias.double(), stride=s, padding=1)
        mag = F.conv2d(xd.abs(), wb.abs(), None, stride=s, padding=1)
        OH, OW = ref.shape[2:]
        d = torch.device("cuda")
        xh = x.permute(0, 2, 3, 1).contiguous().to(d)
        wdev, bd = w.contiguous().to(d), bias.to(d)
        y = torch.full((NF, OH, OW, Co), float("nan"), device=d, dtype=torch.bfloat16)
        wf = torch.empty(2 * 9 * Ci * Co, device=d)  # fp32 image + its bf16 copy
        wd = torch.empty(2 * 9 * Ci * Co, device=d)
        parts = torch.empty((NF * OH * OW // 64 + 2) * 2 * Co, device=d)
        st = nat.stream_of(d)
        nat.check(lib.vad_conv3x3_forward(xh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), bd.data_ptr(), Co, s,
                                          y.data_ptr(), wf.data_ptr(), wd.data_ptr(), parts.data_ptr(), st))
        torch.cuda.synchronize()
        yc = y.cpu().permute(0, 3, 1, 2).double()
        assert torch.isfinite(yc).all()
        bad = (yc - ref).abs() > 2.0 ** -8 * ref.abs() + 1e-5 * mag
        assert not bool(bad.any()), f"forward: {int(bad.sum())} elements outside the bf16 bound"
        dy = torch.randn(NF, Co, OH, OW, generator=g).bfloat16()
        dyd = dy.double()
        dyh = dy.permute(0, 2, 3, 1).contiguous().to(d)
        dx = torch.full((NF, IH, IW, Ci), float("nan"), device=d, dtype=torch.bfloat16)
        nat.check(lib.vad_conv3x3_dgrad(dyh.data_ptr(), NF, Ci, IH, IW, wdev.data_ptr(), Co, s, dx.data_ptr(),
                                        wf.data_ptr(), wd.data_ptr(), st))
        torch.cuda.synchronize()
        rdx = torch.nn.grad.conv2d_input(x.shape, wb, dyd, stride=s, padding=1)
        mdx = torch.nn.grad.conv2d_input(x.shape, wb.abs(), dyd.abs(), stride=s, padding=1)
        dxc = dx.cpu().permute(0, 3, 1, 2).double()
        assert torch.isfinite(dxc).all()
        bad = (dxc - rdx).abs() > 2.0 ** -8 * rdx.abs() + 1e-5 * mdx
        assert not bool(bad.any()), f"input gradient: {int(bad.sum())} elements outside the bf16 bound"
        dW = torch.empty(Co, Ci, 3, 3, device=d)
        part = torch.empty(1 << 24, device=d)
        nat.check(lib.vad_conv3x3_wgrad(xh.data_ptr(), dyh.data_ptr(), NF, Ci, IH, IW, Co, s, dW.data_ptr(),
                                        part.data_ptr(), part.numel(), st))
        torch.cuda.synchronize()
        rdw = torch.nn.grad.conv2d_weight(xd, w.shape, dyd, stride=s, padding=1)
        mdw = torch.nn.grad.conv2d_weight(xd.abs(), w.shape, dyd.abs(), stride=s, padding=1)
        assert float(((dW.cpu().double() - rdw).abs() / (mdw + 1e-30)).max()) < 1e-5
    finally:
        lib.vad_set_tuning(b"act_bf16", 0)
        lib.vad_set_tuning(b"conv_bf16", 0)


@pytest.mark.parametrize("NF,Ci,Co,IH,IW,s", [(8, 32, 32, 57, 57, 1), (6, 128, 128, 15, 15, 1), (8, 32, 64, 57, 57, 2),
                                              (8, 128, 256, 15, 15, 2)])
def test_conv3x3_wgrad_tr_prefetch_is_bit_identical(NF, Ci, Co, IH, IW, s):
    """The transposed-read weight gradient with the next tap's input fragments read before this tap's MFMAs (knob
    conv_wgrad_tr_pft = 1, off by default) computes the same products in the same order: bit-identical dW."""
    nat = _lib()
    _wgrad_path(nat, 3)
    g = torch.Generator().manual_seed(NF + Ci + Co + IH + s)
    d = torch.device("cuda")
    xh = torch.randn(NF, IH, IW, Ci, generator=g).to(d)
    OH, OW = (IH - 1) // s + 1, (IW - 1) // s + 1
    dyh = torch.randn(NF, OH, OW, Co, generator=g).to(d)
    part = torch.empty(1 << 24, device=d)
    out = []
    for pft in (0, 1):
        nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr_pft", pft))
        try:
            dW = torch.empty(Co, Ci, 3, 3, device=d)
            nat.check(nat.lib().vad_conv3x3_wgrad(xh.data_ptr(), dyh.data_ptr(), NF, Ci, IH, IW, Co, s, dW.data_ptr(),
                                                  part.data_ptr(), part.numel(), nat.stream_of(d)))
            torch.cuda.synchronize()
            out.append(dW.cpu())
        finally:
            nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr_pft", 0))
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("bf", [False, True])
@pytest.mark.parametrize("M,C", [(128 * 57 * 57, 32), (7 * 29 * 29 + 3, 64), (128 * 8 * 8, 256), (5, 128)])
def test_bn_bwd_apply_matches_formula(M, C, bf):
    """The BN-backward apply pass alone (vad_bn_bwd_apply; fp32 = config 2, bf16 storage = config 4) against the
    BatchNorm2d + ReLU backward formula in float64 (cad:116,131,136): dY = k (dZ - mean dZ - xhat mean(dZ xhat)),
    dZ = dA [s y + t > 0]; fp32 within a few ulps, bf16 within one bf16 rounding of the output."""
    nat = _lib()
    g = torch.Generator().manual_seed(M + C + bf)
    dt = torch.bfloat16 if bf else torch.float32
    dA = torch.randn(M, C, generator=g).to(dt)
    y = torch.randn(M, C, generator=g).to(dt)
    mean, inv = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    sc, sh, k = torch.randn(C, generator=g), torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g)
    mdz, mdzx = torch.randn(C, generator=g) * 1e-2, torch.randn(C, generator=g) * 1e-2
    stats = torch.cat([mean, inv, sc, sh, k, mdz, mdzx])
    d = torch.device("cuda")
    dY = torch.full((M, C), float("nan"), device=d, dtype=dt)
    dAd, yd = dA.to(d), y.to(d)
    nat.check(nat.lib().vad_bn_bwd_apply(dAd.data_ptr(), yd.data_ptr(), stats.to(d).data_ptr(), M, C, dY.data_ptr(),
                                         1 if bf else 0, nat.stream_of(d)))
    torch.cuda.synchronize()
    a, yy = dA.double(), y.double()
    z = yy * sc.double() + sh.double()
    dz = torch.where(z > 0, a, torch.zeros_like(a))
    xh = (yy - mean.double()) * inv.double()
    ref = k.double() * (dz - mdz.double() - xh * mdzx.double())
    out = dY.cpu().double()
    # error bound: fp32 rounding of each term (mag = the terms' magnitudes; the sum may cancel) + for bf16 storage the
    # output's own rounding; a ReLU decision within rounding of 0 may go either way: those elements are excluded
    mag = k.double().abs() * (dz.abs() + mdz.double().abs() + xh.abs() * mdzx.double().abs())
    keep = (z.abs() > 1e-5)
    bound = 1e-6 * mag + (2.0 ** -8 * ref.abs() if bf else 0.0)
    assert torch.isfinite(out).all()
    bad = ((out - ref).abs() > bound) & keep
    assert not bool(bad.any()), float(((out - ref).abs() - bound)[keep].max())

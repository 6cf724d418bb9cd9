"""Host data path: dataset enumeration + labels against the reference's own constructors
(tests/golden/dataset_enum.json, made by tests/golden/make_dataset_golden.py), the native u8 resize against a
numpy restatement of the same fixed-point bilinear scheme, and (GPU) the pinned staging + u8 -> fp32 kernel.

The resize restates cv2.resize INTER_LINEAR's published u8 algorithm; cv2 is absent here, so beyond the identity
case (UCSD Ped2's native 360x240 frames) it is parity unpinned against cv2 itself."""
import json
import os

import numpy as np
import pytest
import torch

from tests.golden.cases import build_dataset_tree

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dataset_enum.json")))


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("frames"))
    build_dataset_tree(root, empty=False, frame_hw=(24, 36))
    return root


@pytest.mark.parametrize("split", ["Train", "Test"])
def test_cad_clip_enumeration_and_labels_match_reference(tree, split):
    from vad_amd.data import FrameFolderClips
    d = FrameFolderClips(tree, split=split, sequence_length=16, frame_size=(24, 36))
    g = GOLD["cad"][split]
    assert [[os.path.basename(f), names, i] for f, names, i in d.sequences] == g["sequences"]
    assert d.labels == g["labels"]
    x, y = d[len(d) - 1]
    assert x.dtype == torch.uint8 and tuple(x.shape) == (16, 1, 24, 36) and y.dtype == torch.long


@pytest.mark.parametrize("split", ["Train", "Test"])
def test_mc_clip_enumeration_and_labels_match_reference(tree, split):
    from vad_amd.data import FrameFolderClipsMC
    d = FrameFolderClipsMC(tree, subset=split, temporal_frames=8, spatial_size=64, max_clips_per_video=10, stride=4)
    g = GOLD["mc"][split]
    assert [[os.path.relpath(p, tree) for p in c] for c in d.video_clips] == g["clips"]
    assert d.labels == g["labels"]
    x, y = d[0]
    assert x.dtype == torch.uint8 and tuple(x.shape) == (1, 8, 64, 64) and y.dtype == torch.float32


def test_frames_decode_exactly_at_native_size(tree):
    from PIL import Image
    from vad_amd.data import FrameFolderClips
    d = FrameFolderClips(tree, split="Test", sequence_length=16, frame_size=(24, 36))
    folder, names, _ = d.sequences[3]
    x, _ = d[3]
    for t, n in enumerate(names):
        np.testing.assert_array_equal(x[t, 0].numpy(), np.asarray(Image.open(os.path.join(folder, n))))


def _resize_ref(src, dh, dw):
    """numpy restatement of the fixed-point bilinear (half-pixel centres, clamped borders, 11-bit weights)."""
    sh, sw = src.shape

    def table(dn, sn):
        f = ((np.arange(dn) + 0.5) * (sn / dn) - 0.5).astype(np.float32)
        s = np.floor(f).astype(np.int64)
        f = (f - s).astype(np.float32)
        lo, hi = s < 0, s >= sn - 1
        f[lo | hi] = 0
        s[lo] = 0
        s[hi] = sn - 1
        return s, np.rint((1 - f) * 2048).astype(np.int64), np.rint(f * 2048).astype(np.int64)

    xo, xa, xb = table(dw, sw)
    yo, ya, yb = table(dh, sh)
    s = src.astype(np.int64)
    nxt = np.minimum(xo + 1, sw - 1)
    rows = np.where(xo + 1 < sw, s[:, xo] * xa + s[:, nxt] * xb, s[:, xo] * 2048)
    r0, r1 = rows[yo], rows[np.minimum(yo + 1, sh - 1)]
    v = (ya[:, None] * r0 + yb[:, None] * r1 + (1 << 21)) >> 22
    return np.clip(v, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape", [((240, 360), (240, 360)), ((360, 640), (240, 360)), ((57, 91), (64, 64)),
                                   ((64, 64), (227, 227)), ((1, 5), (3, 7))])
def test_native_resize_matches_restatement(shape):
    from vad_amd.data import resize_u8
    (sh, sw), (dh, dw) = shape
    src = np.random.default_rng(sh * dw).integers(0, 256, size=(sh, sw), dtype=np.uint8)
    out = resize_u8(src, dh, dw)
    np.testing.assert_array_equal(out, _resize_ref(src, dh, dw))
    if (sh, sw) == (dh, dw):
        np.testing.assert_array_equal(out, src)


def test_native_resize_constant_and_ramp():
    from vad_amd.data import resize_u8
    np.testing.assert_array_equal(resize_u8(np.full((30, 50), 77, np.uint8), 17, 23), np.full((17, 23), 77))
    ramp = np.tile((np.arange(100) * 2).astype(np.uint8), (10, 1))  # linear in x: preserved inside the image
    out = resize_u8(ramp, 10, 50)
    interior = out[:, 1:-1].astype(int)
    want = np.rint(((np.arange(50) + 0.5) * 2 - 0.5) * 2)[1:-1]
    assert np.abs(interior - want[None, :]).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("pinned", [False, True])
def test_stager_u8_to_clip_bitexact_and_ordered(mode, direct, pinned):
    """prefetch through the stager: every clip bit-equal to the host normalisation, in order; pageable batches through
    the pinned ring, pinned ones read in place; direct (PCIe reads in the conversion kernel) and copy-engine modes;
    odd pixel counts exercise the kernel's per-pixel tail"""
    from vad_amd.data import ClipStager, prefetch
    g = torch.Generator().manual_seed(mode)
    shapes = [(2, 16, 1, 24, 37), (1, 3, 1, 7, 5), (2, 16, 1, 24, 37), (3, 2, 1, 11, 13), (2, 16, 1, 24, 37)]
    batches = [(torch.randint(0, 256, sh, generator=g, dtype=torch.uint8), torch.tensor([i, i]))
               for i, sh in enumerate(shapes)]
    if pinned:
        batches = [(x.pin_memory(), y) for x, y in batches]
    st = ClipStager("cuda", mode=mode, depth=2, direct=direct)
    seen = []
    for (x, y), (xs, ys) in zip(prefetch(batches, st), batches):
        f = xs.float()
        want = (f - 0.5) / 0.5 if mode == 0 else f / 255.0
        np.testing.assert_array_equal(x.cpu().numpy(), want.numpy())
        seen.append(int(y[0]))
    assert seen == list(range(5))


@pytest.mark.gpu
@pytest.mark.parametrize("early", [1, 0])
def test_stager_unwaited_inputs_train_like_staged(early):
    """CadTrainer.step(x, y, inputs_ready=handle.ready) on clips from ClipStager.finish(h, wait=False) -- the step's
    stream never waits for the conversion, the stem does (early stem on; with it off, the armed forward's stem on the
    critical stream) -- gives bit-identical losses and weights to synchronously staged clips"""
    import contextlib
    import io
    from vad_amd import _native as nat
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.data import ClipStager
    from vad_amd.train import CadTrainer, apply_memory_efficient_training
    g = torch.Generator().manual_seed(5)
    u8 = [torch.randint(0, 256, (2, 4, 1, 64, 64), generator=g, dtype=torch.uint8).pin_memory() for _ in range(4)]
    labels = torch.tensor([0, 1], device="cuda")
    res = []
    nat.check(nat.lib().vad_set_tuning(b"cad_stem_early", early))
    try:
        for unwaited in (False, True):
            torch.manual_seed(0)
            m = CausalAnomalyDetector()
            with contextlib.redirect_stdout(io.StringIO()):
                apply_memory_efficient_training(m)
            tr = CadTrainer(m.cuda(), lr=3e-4, seed=11)
            st = ClipStager("cuda", mode=0)
            h = st.issue(u8[0])
            losses = []
            for i in range(4):
                x = st.finish(h, wait=not unwaited)
                ready = h.ready
                if i + 1 < 4:
                    h = st.issue(u8[i + 1])
                if unwaited:
                    losses.append(tr.step(x, labels, inputs_ready=ready).clone())
                else:
                    losses.append(tr.step(x, labels).clone())
            torch.cuda.synchronize()
            res.append((torch.stack(losses).cpu(), {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}))
    finally:
        nat.check(nat.lib().vad_set_tuning(b"cad_stem_early", 1))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)
    for k in res[0][1]:
        torch.testing.assert_close(res[0][1][k], res[1][1][k], rtol=0, atol=0, msg=k)


@pytest.mark.gpu
def test_train_model_on_u8_frame_folders_equals_float_clips(tree):
    """train_model / test_model / evaluate_auc on the u8 frame-folder dataset (staged + normalised on the device)
    give the same weights, losses and scores as on the host-normalised fp32 clips of the reference's pipeline."""
    import contextlib
    import io
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.data import FrameFolderClips
    from vad_amd.evaluate import evaluate_auc
    from vad_amd.train import train_model

    ds = FrameFolderClips(tree, split="Test", sequence_length=4, frame_size=(64, 64))
    sub = torch.utils.data.Subset(ds, list(range(6)))

    class AsFloat(torch.utils.data.Dataset):  # the reference's host path: Normalize(0.5, 0.5) on float frames
        def __len__(self):
            return len(sub)

        def __getitem__(self, i):
            x, y = sub[i]
            return (x.float() - 0.5) / 0.5, y

    res = []
    for data in (sub, AsFloat()):
        torch.manual_seed(0)
        m = CausalAnomalyDetector().cuda()
        tl = torch.utils.data.DataLoader(data, batch_size=2, shuffle=False)
        vl = torch.utils.data.DataLoader(data, batch_size=3, shuffle=False)
        with contextlib.redirect_stdout(io.StringIO()):
            m, tr, va = train_model(m, tl, vl, num_epochs=1, lr=3e-4)
        auc, scores, labels = evaluate_auc(m, vl)
        res.append((torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()]), tr, va, scores))
    np.testing.assert_array_equal(res[0][0].numpy(), res[1][0].numpy())
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
    np.testing.assert_array_equal(res[0][3], res[1][3])
    assert np.isfinite(res[0][1][0])


@pytest.mark.gpu
def test_train_epoch_host_losses_equal_device_losses():
    """train_model's inner loop (train_epoch: prefetch with ready events, the early stem waiting for them, the losses
    read through pinned memory right after each forward) gives the same per-step losses and weights as serial steps
    on synchronously staged clips whose losses are read from the device after each whole step."""
    import contextlib
    import io
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.data import ClipStager
    from vad_amd.train import CadTrainer, apply_memory_efficient_training, train_epoch
    g = torch.Generator().manual_seed(9)
    batches = [(torch.randint(0, 256, (2, 4, 1, 64, 64), generator=g, dtype=torch.uint8), torch.tensor([i % 2, 1]))
               for i in range(5)]
    res = []
    for loop in (False, True):
        torch.manual_seed(0)
        m = CausalAnomalyDetector()
        with contextlib.redirect_stdout(io.StringIO()):
            apply_memory_efficient_training(m)
        tr = CadTrainer(m.cuda(), lr=3e-4, seed=3)
        st = ClipStager("cuda", mode=0)
        per_step = []
        if loop:
            logs = []
            tot, nb = train_epoch(tr, batches, st, lr=2e-4, log=logs.append)
            assert nb == 5 and len(logs) == 1
        else:
            tot, nb = 0.0, 0
            for x, y in batches:
                l = tr.step(st.stage(x), y.cuda(), lr=2e-4).tolist()  # (device losses after the whole step)
                per_step.append(l)
                tot += l[4]
                nb += 1
        torch.cuda.synchronize()
        res.append((tot, torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()])))
        if not loop:
            # host_losses on its own: the same vector as the device's, read after the forward only
            torch.manual_seed(0)
            m2 = CausalAnomalyDetector()
            with contextlib.redirect_stdout(io.StringIO()):
                apply_memory_efficient_training(m2)
            tr2 = CadTrainer(m2.cuda(), lr=3e-4, seed=3)
            for (x, y), want in zip(batches, per_step):
                got = tr2.step(st.stage(x), y.cuda(), lr=2e-4, host_losses=True)
                assert got.device.type == "cpu" and got.tolist() == want
    assert res[0][0] == res[1][0]
    np.testing.assert_array_equal(res[0][1].numpy(), res[1][1].numpy())

"""Host data path of the training loop: frame folders -> u8 clips -> pinned staging -> HBM.

The reference decodes every frame with cv2/PIL into float tensors on the host (UCSDped2Dataset.__getitem__,
causal_anomaly_detection.py:85-104; UCSDped2SimpleDataset, minicausal_vad_complete3.py:192-216) and copies fp32
clips to the device inside the step (cad:639, mc:266).  Here the loader keeps clips as **u8** end to end:

* ``FrameFolderClips`` / ``FrameFolderClipsMC`` enumerate the same overlapping clips with the same (synthesised)
  labels as the reference datasets (cad:39-80, mc:104-190) and return ``(T, 1, H, W)`` / ``(1, T, H, W)`` uint8
  frames; decoding is PIL, resizing the native ``vad_resize_u8`` (cv2 INTER_LINEAR scheme, cad:88-89).
* ``ClipStager`` keeps u8 batches in pinned host memory, copies them to the device as u8 and converts them to fp32
  there (``vad_u8_to_clip``: the reference's Normalize(0.5, 0.5) over raw 0..255 pixels, or ToTensor's /255), both
  on a stream of its own -- a quarter of the PCIe bytes of fp32 clips, and batch k+1's staging overlaps step k.
* ``prefetch(loader, stager)`` yields device clips one batch ahead.
"""
from __future__ import annotations

import ctypes
import os
import random

import numpy as np
import torch

from . import _native as nat

_EXTS_CAD = (".jpg", ".png", ".tif")


def _decode_gray(path: str, size_hw: tuple[int, int] | None, pil_resize: bool = False) -> np.ndarray:
    """One frame as (H, W) uint8 grayscale (PIL's ITU-R 601 luma for colour frames), resized to size_hw when given:
    cad: cv2.imread GRAYSCALE + cv2.resize (cad:87-88) -> the native bilinear; mc: PIL + torchvision Resize, which
    is PIL's own bilinear resize (mc:117-119) -> pil_resize=True."""
    from PIL import Image
    with Image.open(path) as im:
        g = im.convert("L")
        if pil_resize and size_hw is not None and g.size != (size_hw[1], size_hw[0]):
            g = g.resize((size_hw[1], size_hw[0]), Image.BILINEAR)
        a = np.asarray(g, dtype=np.uint8)
    if size_hw is not None and a.shape != tuple(size_hw):
        return resize_u8(a, *size_hw)
    return np.ascontiguousarray(a)


def resize_u8(img: np.ndarray, h: int, w: int) -> np.ndarray:
    """Bilinear resize of a (H, W) uint8 image (native vad_resize_u8)."""
    src = np.ascontiguousarray(img, dtype=np.uint8)
    dst = np.empty((h, w), dtype=np.uint8)
    nat.check(nat.lib().vad_resize_u8(src.ctypes.data, src.shape[0], src.shape[1], dst.ctypes.data, h, w))
    return dst


class FrameFolderClips(torch.utils.data.Dataset):
    """UCSDped2Dataset (cad:39-104): clips of ``sequence_length`` frames with stride sequence_length // 2 over every
    frame folder of ``root/split``; Train labels 0, Test labels from the reference's heuristic (cad:62-80, the same
    ``random.seed(folder_num * 1000 + i)`` draw).  Items: ((T, 1, 240, 360) uint8, int64 label)."""

    def __init__(self, root_dir, split="Train", sequence_length=16, frame_size=(240, 360)):
        self.root_dir = os.path.join(root_dir, split)
        self.sequence_length = sequence_length
        self.frame_size = frame_size
        self.sequences, self.labels = [], []
        T = sequence_length
        for folder in sorted(os.listdir(self.root_dir)):
            folder_path = os.path.join(self.root_dir, folder)
            if not os.path.isdir(folder_path):
                continue
            frames = sorted(f for f in os.listdir(folder_path) if f.endswith(_EXTS_CAD))
            for i in range(0, len(frames) - T + 1, T // 2):
                seq = frames[i:i + T]
                if len(seq) != T:
                    continue
                self.sequences.append((folder_path, seq, i))
                if split == "Train":
                    self.labels.append(0)
                    continue
                folder_num = int(folder.replace("Test", "").replace("Train", ""))
                progress = i / max(len(frames) - T, 1)
                p = 0.0
                if folder_num in (1, 3, 5, 7, 9, 11):
                    p += 0.4
                if progress > 0.6:
                    p += 0.3
                if 0.3 < progress < 0.7:
                    p += 0.2
                rnd = random.Random(folder_num * 1000 + i)  # == random.seed(...); random.random() (cad:78-79)
                self.labels.append(1 if rnd.random() < p else 0)

    def __len__(self):
        return len(self.sequences)

    def __getitem__(self, idx):
        folder_path, names, _ = self.sequences[idx]
        frames = np.stack([_decode_gray(os.path.join(folder_path, n), self.frame_size) for n in names])
        return torch.from_numpy(frames).unsqueeze(1), torch.tensor(self.labels[idx], dtype=torch.long)


class FrameFolderClipsMC(torch.utils.data.Dataset):
    """UCSDped2SimpleDataset (mc:104-216): .tif folders (``*_gt`` skipped), clips of ``temporal_frames`` at
    ``stride``, at most ``max_clips_per_video`` per video, the reference's label rule (mc:165-172).  Items:
    ((1, T, S, S) uint8, float32 label); the device conversion is ToTensor's /255 (mode 1)."""

    def __init__(self, root_dir, subset="Train", temporal_frames=8, spatial_size=64, max_clips_per_video=10,
                 stride=4):
        self.spatial_size = spatial_size
        self.video_clips, self.labels = [], []
        subset_path = os.path.join(root_dir, subset)
        if not os.path.exists(subset_path):
            raise ValueError(f"Path {subset_path} does not exist")
        folders = sorted(f for f in os.listdir(subset_path)
                         if os.path.isdir(os.path.join(subset_path, f)) and not f.endswith("_gt"))
        for video_idx, folder in enumerate(folders):
            vp = os.path.join(subset_path, folder)
            files = sorted(f for f in os.listdir(vp) if f.endswith(".tif"))
            if len(files) < temporal_frames:
                continue
            added = 0
            for start in range(0, len(files) - temporal_frames + 1, stride):
                if added >= max_clips_per_video:
                    break
                self.video_clips.append([os.path.join(vp, f) for f in files[start:start + temporal_frames]])
                label = (1 if (video_idx * added) % 5 == 0 else 0) if subset == "Train" else (1 if added % 2 == 0
                                                                                               else 0)
                self.labels.append(label)
                added += 1
        if len(set(self.labels)) < 2:
            # the reference's forced anomalies (mc:176-183): the same draw from numpy's global generator
            normal = [i for i, l in enumerate(self.labels) if l == 0]
            if normal:
                for i in np.random.choice(normal, min(len(normal) // 3, 10), replace=False):
                    self.labels[i] = 1

    def __len__(self):
        return len(self.video_clips)

    def __getitem__(self, idx):
        S = self.spatial_size
        frames = np.stack([_decode_gray(p, (S, S), pil_resize=True) for p in self.video_clips[idx]])
        return torch.from_numpy(frames).unsqueeze(0), torch.tensor(float(self.labels[idx]), dtype=torch.float32)


class _Staged:
    """An issued batch: its fp32 device clip (being written on the stager's stream) and the event that completes it."""
    __slots__ = ("out", "ready", "slot")

    def __init__(self, out, ready, slot):
        self.out, self.ready, self.slot = out, ready, slot


class ClipStager:
    """Pinned u8 staging + on-device u8 -> fp32 conversion on a stream of its own, one batch ahead of the step.

    ``issue(batch_u8)`` enqueues batch k+1's conversion while step k computes and returns a handle; ``finish(handle)``
    returns its fp32 device clip, ordered on the current stream (``wait=True``) or left to the consumer
    (``wait=False``: hand ``handle.ready`` to ``CadTrainer.step(inputs_ready=...)``, whose early stem waits for it on
    the plan's stem stream and the step's critical stream never does).  ``stage(batch)`` = ``finish(issue(batch))``.
    mode 0: (u8 - 0.5) / 0.5 (cad), 1: u8 / 255 (mc/bbox).

    direct=False (default): an H2D copy of the u8 batch into a device buffer (the copy engine), then the conversion,
    both on the stager's stream.  Nothing queued there waits for the step's streams: the u8 and fp32 device buffers
    are stream-ordered by the caching allocator (the fp32 clip recorded on its consumer's stream), which matters --
    HIP spreads streams over GPU_MAX_HW_QUEUES (4) hardware queues, and the previous design (a fixed device slot whose
    copy waited for an event of the step's stream) stalled whichever step stream shared the copy's queue: config 2 at
    3.0 ms/step on two of the four queues, 1.80 on the others; this one 1.75-1.83 ms on all four against 1.74 ms with
    clips already in HBM (profiles/r04_h2d_queues.json).  direct=True: the conversion kernel reads the pinned host
    batch itself over PCIe (``vad_host_device_ptr``), no copy engine and no u8 device buffer (1.86-1.93 ms: the
    PCIe-bound kernel holds CUs beside the step).

    A batch that is not pinned and contiguous goes through a ring of ``depth`` pinned buffers (a slot is refilled
    once its previous conversion has finished); a pinned batch is read in place and must not be overwritten until
    ``handle.ready`` has completed.  Each returned clip is a fresh tensor (recorded on the consuming stream)."""

    def __init__(self, device, mode=0, depth=2, direct=False):
        self.device = torch.device(device)
        nat.require_hip(torch.empty(0, device=self.device))
        self.mode = mode
        self.depth = depth
        self.direct = direct
        self.stream = torch.cuda.Stream(self.device)
        self.copy_stream = self.stream  # (the name of earlier releases)
        self._ring = []  # [pinned u8, device u8 (direct=False), conversion-done event]
        self._k = 0
        self._dptr = {}  # pinned host pointer -> its device address
        # direct mode: caller-owned pinned batches read in place over PCIe, kept alive until their conversion is done
        # (the caching host allocator records no event for a kernel's reads, so a dropped batch could be reused, e.g.
        # by a DataLoader pin thread, while the conversion still reads it)
        self._inflight = []

    def _slot(self, shape):
        if len(self._ring) <= self._k or tuple(self._ring[self._k][0].shape) != tuple(shape):
            slot = [torch.empty(shape, dtype=torch.uint8, pin_memory=True), None, torch.cuda.Event()]
            if len(self._ring) <= self._k:
                self._ring.append(slot)
            else:
                # (a shape change, e.g. the last partial batch: the old pinned buffer may still be read by its
                # conversion -- direct mode reads it over PCIe, with no host-allocator event -- before it is freed)
                self._ring[self._k][2].synchronize()
                self._ring[self._k] = slot
        return self._ring[self._k]

    def _device_address(self, host: torch.Tensor) -> int:
        p = host.data_ptr()
        d = self._dptr.get(p)
        if d is None:
            out = ctypes.c_void_p()
            nat.check(nat.lib().vad_host_device_ptr(p, ctypes.addressof(out)))
            d = self._dptr[p] = out.value
            if len(self._dptr) > 64:  # (caller-owned pinned batches come and go)
                self._dptr.pop(next(iter(self._dptr)))
        return d

    def issue(self, batch_u8: torch.Tensor) -> _Staged:
        """Enqueue one u8 batch's conversion (and, direct=False, its H2D copy) on the stager's stream."""
        if batch_u8.dtype != torch.uint8:
            raise TypeError("ClipStager.issue expects a uint8 batch")
        if batch_u8.numel() == 0:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            return _Staged(torch.empty(batch_u8.shape, dtype=torch.float32, device=self.device), ev, None)
        if batch_u8.is_pinned() and batch_u8.is_contiguous() and batch_u8.data_ptr() % 16 == 0:
            src, slot, done = batch_u8, None, torch.cuda.Event()
        else:
            slot = self._slot(batch_u8.shape)
            self._k = (self._k + 1) % self.depth
            src, done = slot[0], slot[2]
            done.synchronize()  # the slot's previous conversion (or copy) has read the pinned buffer
            src.copy_(batch_u8)
        with torch.cuda.stream(self.stream):
            out = torch.empty(batch_u8.shape, dtype=torch.float32, device=self.device)
            if self.direct:
                sp = self._device_address(src)
            else:
                dev = torch.empty(batch_u8.shape, dtype=torch.uint8, device=self.device)
                dev.copy_(src, non_blocking=True)
                sp = dev.data_ptr()
            nat.check(nat.lib().vad_u8_to_clip(sp, src.numel(), self.mode, out.data_ptr(),
                                               ctypes.c_void_p(self.stream.cuda_stream)))
            done.record(self.stream)
        if self.direct and slot is None:
            self._inflight = [(b, e) for b, e in self._inflight if not e.query()]
            self._inflight.append((src, done))
        return _Staged(out, done, slot)

    def finish(self, handle: _Staged, wait: bool = True) -> torch.Tensor:
        """The fp32 device clip of an issued batch.  wait=True: ready on the current stream; wait=False: the consumer
        orders itself after ``handle.ready`` (e.g. CadTrainer.step(x, y, inputs_ready=handle.ready))."""
        cur = torch.cuda.current_stream(self.device)
        if wait:
            cur.wait_event(handle.ready)
        handle.out.record_stream(cur)  # (its memory is not reused before the current stream's queued work is done)
        return handle.out

    def stage(self, batch_u8: torch.Tensor) -> torch.Tensor:
        return self.finish(self.issue(batch_u8))


def prefetch(loader, stager: ClipStager, with_ready: bool = False):
    """Iterate (device clips, device labels) one batch ahead: the H2D copy of batch k+1 is issued before batch k is
    yielded (it runs on the copy stream while step k computes) and converted when batch k+1 is yielded.  uint8
    batches go through the stager; float batches (the reference's own datasets) are copied as they are.
    with_ready=True: yields (clips, labels, ready) -- for a staged batch the current stream does not wait for it and
    ``ready`` is the event that completes it (hand it to CadTrainer.step(inputs_ready=...)); None otherwise."""
    def issue(x, y):
        h = stager.issue(x) if x.dtype == torch.uint8 else x
        return h, y

    def finish(h, y):
        yd = y.to(stager.device, non_blocking=True)
        if isinstance(h, torch.Tensor):
            xd = h.to(stager.device, non_blocking=True)
            return (xd, yd, None) if with_ready else (xd, yd)
        if with_ready:
            return stager.finish(h, wait=False), yd, h.ready
        return stager.finish(h), yd

    it = iter(loader)
    try:
        pending = issue(*next(it))
    except StopIteration:
        return
    for x, y in it:
        cur = finish(*pending)
        pending = issue(x, y)
        yield cur
    yield finish(*pending)

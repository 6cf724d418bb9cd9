"""Host data path of the training loop: frame folders -> u8 clips -> pinned staging -> HBM.

The reference decodes every frame with cv2/PIL into float tensors on the host (UCSDped2Dataset.__getitem__,
causal_anomaly_detection.py:85-104; UCSDped2SimpleDataset, minicausal_vad_complete3.py:192-216) and copies fp32
clips to the device inside the step (cad:639, mc:266).  Here the loader keeps clips as **u8** end to end:

* ``FrameFolderClips`` / ``FrameFolderClipsMC`` enumerate the same overlapping clips with the same (synthesised)
  labels as the reference datasets (cad:39-80, mc:104-190) and return ``(T, 1, H, W)`` / ``(1, T, H, W)`` uint8
  frames; decoding is PIL, resizing the native ``vad_resize_u8`` (cv2 INTER_LINEAR scheme, cad:88-89).
* ``ClipStager`` copies a u8 batch into a ring of pinned host buffers, issues the host-to-device copy on its own
  HIP stream and converts u8 -> fp32 on the device (``vad_u8_to_clip``: the reference's Normalize(0.5, 0.5) over
  raw 0..255 pixels, or ToTensor's /255) -- a quarter of the PCIe bytes of fp32 clips, and the copy of batch k+1
  overlaps step k.
* ``prefetch(loader, stager)`` yields device clips one batch ahead.
"""
from __future__ import annotations

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


class ClipStager:
    """Pinned u8 staging ring + H2D copies on a dedicated stream + on-device u8 -> fp32 conversion.

    Two halves, so the copy of batch k+1 overlaps step k: ``issue(batch_u8)`` puts the batch into a pinned ring slot
    (skipped when the batch is already pinned) and enqueues its H2D copy on the copy stream, ordered only after the
    previous conversion out of the same device slot (not after the compute stream's other work); ``finish(handle)``
    makes the current stream wait for that copy and converts it to the fp32 device clip.  ``stage(batch)`` =
    ``finish(issue(batch))``.  mode 0: (u8 - 0.5) / 0.5 (cad), 1: u8 / 255 (mc/bbox)."""

    def __init__(self, device, mode=0, depth=2):
        self.device = torch.device(device)
        nat.require_hip(torch.empty(0, device=self.device))
        self.mode = mode
        self.depth = depth
        self.copy_stream = torch.cuda.Stream(self.device)
        self._ring = []  # [pinned u8, device u8, copy-done event, read-done event]
        self._k = 0

    def _slot(self, shape):
        if len(self._ring) <= self._k or tuple(self._ring[self._k][0].shape) != tuple(shape):
            slot = [torch.empty(shape, dtype=torch.uint8, pin_memory=True),
                    torch.empty(shape, dtype=torch.uint8, device=self.device), torch.cuda.Event(), torch.cuda.Event()]
            if len(self._ring) <= self._k:
                self._ring.append(slot)
            else:
                self._ring[self._k] = slot
        return self._ring[self._k]

    def issue(self, batch_u8: torch.Tensor):
        """Start the H2D copy of one u8 batch; returns the handle for finish()."""
        if batch_u8.dtype != torch.uint8:
            raise TypeError("ClipStager.issue expects a uint8 batch")
        slot = self._slot(batch_u8.shape)
        pinned, dev, copied, read = slot
        if batch_u8.is_pinned():
            src = batch_u8
        else:
            copied.synchronize()  # the previous H2D out of this pinned buffer has finished
            pinned.copy_(batch_u8)
            src = pinned
        self.copy_stream.wait_event(read)  # the previous u8 -> fp32 conversion out of this device slot is done
        with torch.cuda.stream(self.copy_stream):
            dev.copy_(src, non_blocking=True)
            copied.record(self.copy_stream)
        self._k = (self._k + 1) % self.depth
        return slot

    def finish(self, handle) -> torch.Tensor:
        """The fp32 device clip of an issued batch, ready on the current stream."""
        _, dev, copied, read = handle
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(copied)
        out = torch.empty(dev.shape, dtype=torch.float32, device=self.device)
        nat.check(nat.lib().vad_u8_to_clip(dev.data_ptr(), dev.numel(), self.mode, out.data_ptr(),
                                           nat.stream_of(self.device)))
        read.record(cur)
        return out

    def stage(self, batch_u8: torch.Tensor) -> torch.Tensor:
        return self.finish(self.issue(batch_u8))


def prefetch(loader, stager: ClipStager):
    """Iterate (device clips, device labels) one batch ahead: the H2D copy of batch k+1 is issued before batch k is
    yielded (it runs on the copy stream while step k computes) and converted when batch k+1 is yielded.  uint8
    batches go through the stager; float batches (the reference's own datasets) are copied as they are."""
    def issue(x, y):
        h = stager.issue(x) if x.dtype == torch.uint8 else x
        return h, y

    def finish(h, y):
        xd = stager.finish(h) if not isinstance(h, torch.Tensor) else h.to(stager.device, non_blocking=True)
        return xd, y.to(stager.device, non_blocking=True)

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

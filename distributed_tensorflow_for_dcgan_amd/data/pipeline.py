"""Input pipelines: synthetic images, TFRecord files (native threaded loader), image folders.

Replaces ``image_input.distorted_inputs`` (reference ``image_input.py:98-143``) and the
``sess.run(images)`` host round trip of ``image_train.py:153``: batches are produced by the C++
loader straight into pinned host buffers, copied to the GPU asynchronously on a side stream
one or more steps ahead, and handed to the engine as device tensors.

Sharding: with ``shard=True`` rank r of W reads the files ``files[r::W]`` (disjoint) when
there are at least W files; otherwise every rank reads every file with a rank-specific shuffle
seed (the reference behaviour: every worker reads the same files, ``image_input.py:107``).
"""
from __future__ import annotations

import os
import queue
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import tfrecord as TR

NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN = 107766  # reference image_input.py:14
LOADER_DTYPE = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16"}
ENGINE_DTYPE = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


def batch_dtype(device, engine_dtype: Optional[str] = None) -> torch.dtype:
    """The dtype batches are decoded into: the compute dtype of the engine that was BUILT
    (``engine.dtype_name``) on a GPU -- bf16 batches halve the H2D bytes and need no on-device
    cast -- and fp32 on the CPU or when the engine is unknown (the fp32 reference engine must
    never see quantized inputs)."""
    if torch.device(device).type != "cuda" or engine_dtype is None:
        return torch.float32
    return ENGINE_DTYPE.get(str(engine_dtype), torch.float32)


class SyntheticSource:
    """Uniform[-1,1] images of the configured shape, generated on the device."""

    def __init__(self, batch: int, shape: Tuple[int, int, int], device, seed: int = 0, fixed: bool = False,
                 num_examples: int = NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN * 3):
        self.batch, self.shape, self.device = batch, tuple(shape), torch.device(device)
        self.gen = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        self.gen.manual_seed(seed)
        self.fixed = fixed
        self._fixed = None
        self.num_examples = num_examples

    def next(self) -> torch.Tensor:
        if self.fixed and self._fixed is not None:
            return self._fixed
        x = torch.rand((self.batch,) + self.shape, generator=self.gen, device=self.device) * 2 - 1
        if self.fixed:
            self._fixed = x
        return x

    def stats(self):
        return {"source": "synthetic"}

    def close(self):
        pass


def shard_files(files: Sequence[str], rank: int, world: int, shard: bool) -> Tuple[List[str], bool]:
    if shard and world > 1 and len(files) >= world:
        return list(files[rank::world]), True
    return list(files), False


class TFRecordSource:
    """Native threaded TFRecord loader + pinned ring + async H2D."""

    def __init__(self, data_dir: str, batch: int, shape: Tuple[int, int, int], device, rank: int = 0,
                 world: int = 1, shard: bool = True, shuffle_buffer: int = 10776, threads: int = 16, seed: int = 0,
                 out_dtype: str = "f32", loop: bool = True, prefetch: int = 3, feature: str = "image_raw",
                 num_examples: Optional[int] = None):
        from . import native
        files = TR.list_record_files(data_dir)
        self.files, self.sharded = shard_files(files, rank, world, shard)
        self.batch, self.shape = batch, tuple(shape)
        self.device = torch.device(device)
        H, W, C = self.shape
        self.num_examples = num_examples if num_examples is not None else TR.count_records(files)
        cap = shuffle_buffer + 3 * batch  # reference: capacity = min_queue + 3 * batch
        self.loader = native.ext().Loader(self.files, feature, H, W, C, batch, cap, shuffle_buffer, threads,
                                          int(seed) * 1000003 + rank, out_dtype, "auto", loop, True,
                                          1.0 / 127.5, -1.0)
        tdtype = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[out_dtype]
        pin = self.device.type == "cuda"
        self._host = [torch.empty((batch,) + self.shape, dtype=tdtype, pin_memory=pin) for _ in range(prefetch)]
        self._dev = [torch.empty((batch,) + self.shape, dtype=tdtype, device=self.device) for _ in range(prefetch)]
        self._ready: "queue.Queue" = queue.Queue()
        self._free: "queue.Queue" = queue.Queue()
        for i in range(prefetch):
            self._free.put(i)
        self._copied = [None] * prefetch
        self._consumed = [None] * prefetch
        self.copy_stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self._stop = False
        self._err: Optional[BaseException] = None
        self._thread = threading.Thread(target=self._fill, daemon=True)
        self._thread.start()
        self._cur = None

    def _fill(self):
        """Producer thread: native loader -> pinned host buffer -> async H2D on the copy stream.
        A device slot is overwritten only after the compute stream consumed it (event), and a
        pinned buffer only after its previous H2D copy completed."""
        try:
            while not self._stop:
                i = self._free.get()
                if i is None:
                    return
                ev = self._copied[i]
                if ev is not None:
                    ev.synchronize()
                n = self.loader.next_batch(self._host[i].data_ptr())
                if n < self.batch:
                    self._ready.put(None)
                    return
                if self.copy_stream is not None:
                    with torch.cuda.stream(self.copy_stream):
                        if self._consumed[i] is not None:
                            self.copy_stream.wait_event(self._consumed[i])
                        self._dev[i].copy_(self._host[i], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.copy_stream)
                    self._copied[i] = ev
                self._ready.put(i)
        except BaseException as e:  # surfaced on the consumer side
            self._err = e
            self._ready.put(None)

    def next(self) -> torch.Tensor:
        i = self._ready.get()
        if i is None:
            if self._err is not None:
                raise self._err
            raise StopIteration
        if self.copy_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._copied[i])
            out = self._dev[i]
        else:
            out = self._host[i].clone()
        # the previously returned slot is consumed by everything enqueued so far
        if self._cur is not None:
            if self.copy_stream is not None:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                self._consumed[self._cur] = ev
            self._free.put(self._cur)
        self._cur = i
        return out

    def stats(self):
        s = dict(self.loader.stats())
        s["source"] = "tfrecord"
        s["files"] = len(self.files)
        s["sharded"] = self.sharded
        return s

    def close(self):
        self._stop = True
        self.loader.stop()
        self._free.put(None)


class DeviceCachedSource:
    """The whole (sharded) TFRecord dataset decoded ONCE by the native loader and kept in GPU
    memory (``--cache_on_device``; SURVEY.md §7.2 item 8: 64x64x3 CelebA-size data is ~2.5 GB
    in bf16, far below 288 GB of HBM3E). Every epoch is a fresh on-device permutation and a
    batch is one gather kernel: no host work, no H2D copy in the steady state."""

    def __init__(self, data_dir: str, batch: int, shape: Tuple[int, int, int], device, rank: int = 0,
                 world: int = 1, shard: bool = True, seed: int = 0, threads: int = 16,
                 feature: str = "image_raw", dtype: Optional[torch.dtype] = None):
        from . import native
        files = TR.list_record_files(data_dir)
        self.files, self.sharded = shard_files(files, rank, world, shard)
        self.batch, self.shape = batch, tuple(shape)
        self.device = torch.device(device)
        H, W, C = self.shape
        n = TR.count_records(self.files)
        if n < batch:
            raise ValueError("dataset shard has %d examples < batch %d" % (n, batch))
        self.num_examples = TR.count_records(files)
        dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.data = torch.empty((n,) + self.shape, dtype=dtype, device=self.device)
        chunk = max(batch, 256)
        loader = native.ext().Loader(self.files, feature, H, W, C, chunk, chunk, 0, threads, int(seed) + rank,
                                     LOADER_DTYPE[dtype], "auto", False, True, 1.0 / 127.5, -1.0)
        host = torch.empty((chunk,) + self.shape, dtype=dtype, pin_memory=self.device.type == "cuda")
        filled = 0
        try:
            while filled < n:
                got = loader.next_batch(host.data_ptr())
                if got <= 0:
                    break
                got = min(got, n - filled)
                self.data[filled:filled + got].copy_(host[:got])
                filled += got
        finally:
            loader.stop()
        self.data = self.data[:filled]
        self.n = filled
        self.gen = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        self.gen.manual_seed(int(seed) * 7919 + rank)
        self._perm = None
        self._pos = 0

    def next(self) -> torch.Tensor:
        if self._perm is None or self._pos + self.batch > self.n:
            self._perm = torch.randperm(self.n, generator=self.gen, device=self.device)
            self._pos = 0
        idx = self._perm[self._pos:self._pos + self.batch]
        self._pos += self.batch
        return self.data.index_select(0, idx)

    def stats(self):
        return {"source": "device_cache", "examples": self.n, "bytes": self.data.numel() * self.data.element_size()}

    def close(self):
        self.data = None


class ImageFolderSource:
    """PNG/JPEG folder (``--dataset`` directory of images): optional center crop of
    ``image_size`` (``--is_crop``), resize to ``output_size``, scale to [-1, 1]; decoded by a
    small thread pool with PIL. Provided for the carpedm20-style datasets (celebA, lsun dumps)."""

    EXTS = (".png", ".jpg", ".jpeg", ".bmp", ".webp")

    def __init__(self, folder: str, batch: int, shape: Tuple[int, int, int], device, is_crop: bool = False,
                 image_size: int = 108, rank: int = 0, world: int = 1, shard: bool = True, seed: int = 0,
                 threads: int = 8):
        files = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(folder) for f in fs
                       if f.lower().endswith(self.EXTS))
        if not files:
            raise FileNotFoundError("no images in %s" % folder)
        self.files, self.sharded = shard_files(files, rank, world, shard)
        self.batch, self.shape, self.device = batch, tuple(shape), torch.device(device)
        self.is_crop, self.image_size = is_crop, image_size
        self.rng = np.random.default_rng(seed + 7 * rank)
        self.num_examples = len(files)
        from concurrent.futures import ThreadPoolExecutor
        self.pool = ThreadPoolExecutor(max_workers=threads)
        self._order = []

    def _load(self, path: str) -> np.ndarray:
        from PIL import Image
        H, W, C = self.shape
        im = Image.open(path).convert("L" if C == 1 else "RGB")
        if self.is_crop:
            w, h = im.size
            cs = min(self.image_size, w, h)
            l, t = (w - cs) // 2, (h - cs) // 2
            im = im.crop((l, t, l + cs, t + cs))
        im = im.resize((W, H), Image.BICUBIC)
        a = np.asarray(im, dtype=np.float32) / 127.5 - 1.0
        return a.reshape(H, W, C)

    def next(self) -> torch.Tensor:
        if len(self._order) < self.batch:
            self._order += list(self.rng.permutation(len(self.files)))
        idx, self._order = self._order[:self.batch], self._order[self.batch:]
        imgs = list(self.pool.map(self._load, [self.files[i] for i in idx]))
        return torch.from_numpy(np.stack(imgs)).to(self.device, non_blocking=True)

    def stats(self):
        return {"source": "images", "files": len(self.files)}

    def close(self):
        self.pool.shutdown(wait=False)


def make_source(flags, batch: int, shape, device, rank: int = 0, world: int = 1, data_dir: Optional[str] = None,
                seed_offset: int = 0, loop: bool = True, shuffle_buffer: Optional[int] = None,
                engine_dtype: Optional[str] = None):
    """Pick the input source from the flags: --synthetic, a TFRecord directory (reference
    default ``--data_dir=train``), or a folder of images. engine_dtype: the built engine's
    ``dtype_name`` (TFRecord batches are decoded into it on a GPU; fp32 when None)."""
    seed = int(flags.seed) + seed_offset
    if flags.synthetic:
        return SyntheticSource(batch, shape, device, seed=seed + 1000 * rank)
    d = data_dir or flags.data_dir
    if os.path.isdir(d):
        names = os.listdir(d)
        if names and all(n.lower().endswith(ImageFolderSource.EXTS) for n in names if not n.startswith(".")):
            return ImageFolderSource(d, batch, shape, device, is_crop=bool(flags.is_crop),
                                     image_size=int(flags.image_size), rank=rank, world=world,
                                     shard=bool(flags.shard_data), seed=seed)
    dt = batch_dtype(device, engine_dtype)
    if bool(getattr(flags, "cache_on_device", False)) and data_dir is None:
        return DeviceCachedSource(d, batch, shape, device, rank=rank, world=world, shard=bool(flags.shard_data),
                                  seed=seed, threads=int(flags.loader_threads), dtype=dt)
    sb = int(flags.shuffle_buffer) if shuffle_buffer is None else shuffle_buffer
    return TFRecordSource(d, batch, shape, device, rank=rank, world=world, shard=bool(flags.shard_data),
                          shuffle_buffer=sb, threads=int(flags.loader_threads), seed=seed, loop=loop,
                          out_dtype=LOADER_DTYPE[dt])

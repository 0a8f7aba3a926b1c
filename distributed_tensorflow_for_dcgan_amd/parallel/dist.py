"""Synchronous data parallelism: process groups, broadcast, bucketed gradient all-reduce.

Replaces the reference's asynchronous gRPC parameter server (all variables pinned to
``/job:ps/task:0``, ``distriubted_model.py:70``; ``replica_device_setter``,
``image_train.py:65-67``) with one process per GPU and collectives:

* init: ``broadcast`` of every parameter / BN moving average from rank 0 (replaces "the
  PS is the single source of truth");
* per step: gradient ``all_reduce`` (SUM, then x 1/W) over flat per-model buffers, cut
  into buckets so that each bucket's collective can start as soon as its gradients are
  final and overlap with the remaining backward on a separate stream;
* backend ``nccl`` (= RCCL over xGMI on ROCm) for GPUs, ``gloo`` for CPU tests.

RCCL's ring over the 8-GPU xGMI full mesh is per-link bound (~153 GB/s per link), so
buckets are kept large: the HIP engine overlaps at graph-segment granularity (G grads
during D's backward, D's top layer during the rest of D's backward), so each overlap
window is ONE collective (32 MiB buckets) -- extra calls would only add latency.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

_PG_INITIALISED_HERE = False
_NATIVE = None  # native RCCL communicator over the default group's ranks (native_comm)


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def backend() -> Optional[str]:
    """The default process group's backend ("nccl" = RCCL, "gloo"), None without one."""
    return dist.get_backend() if is_initialized() else None


def ddp_forced() -> bool:
    """DCGAN_FORCE_DDP=1: run the data-parallel path (process group, collectives on the comm
    stream, segmented step) even for a single process -- a one-rank RCCL group exercises the
    real collective code on a one-GPU machine."""
    return os.environ.get("DCGAN_FORCE_DDP", "") == "1"


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_distributed(world: int, rank_: int, device: torch.device, master_addr: Optional[str] = None,
                     master_port: Optional[int] = None, timeout_s: float = 600.0, force: Optional[bool] = None):
    """Create the default process group when world > 1, or for one process when forced
    (``force`` / DCGAN_FORCE_DDP=1); otherwise a no-op."""
    global _PG_INITIALISED_HERE
    force = ddp_forced() if force is None else bool(force)
    if (world <= 1 and not force) or is_initialized():
        return dist.group.WORLD if is_initialized() else None
    os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
    if world <= 1 and "MASTER_PORT" not in os.environ and master_port is None:
        os.environ["MASTER_PORT"] = str(_free_port())  # a lone rank: any free port
    os.environ.setdefault("MASTER_PORT", str(master_port or 29500))
    backend = "nccl" if device.type == "cuda" else "gloo"
    # gloo over GPU tensors lets several ranks share ONE GPU (RCCL refuses that): used by the
    # 1-GPU DDP-equivalence test of the HIP engine. Production multi-GPU runs use RCCL.
    backend = os.environ.get("DCGAN_DIST_BACKEND", backend)
    kwargs = dict(backend=backend, world_size=world, rank=rank_,
                  timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kwargs["device_id"] = device
    dist.init_process_group(**kwargs)
    _PG_INITIALISED_HERE = True
    return dist.group.WORLD


def _rccl_path() -> str:
    """The RCCL that PyTorch loaded (its bundled librccl.so): one RCCL per process."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


def native_comm(device: torch.device):
    """A native RCCL communicator (csrc/comm.h) over the default process group's ranks, for the
    gradient all-reduces: ncclAllReduce straight onto the engine's comm stream from C++ -- no
    ProcessGroupNCCL internal stream, event hand-offs or Python call per collective, and
    capturable into a hipGraph. Rank 0 makes the unique id, the process group broadcasts it.
    None without an RCCL ("nccl") group or with DCGAN_NATIVE_RCCL=0 (torch.distributed then
    issues the collectives)."""
    global _NATIVE
    if _NATIVE is None:
        if (not is_initialized() or dist.get_backend() != "nccl" or device.type != "cuda"
                or os.environ.get("DCGAN_NATIVE_RCCL", "1") == "0"):
            return None
        from ..ops import hip as H
        ext = H.ext()
        lib = _rccl_path()
        obj = [ext.RcclComm.unique_id(lib) if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        _NATIVE = ext.RcclComm(lib, dist.get_world_size(), dist.get_rank(), obj[0], device.index or 0)
    return _NATIVE


def shutdown() -> None:
    """Tear down the native communicator and the process group this module created. Every
    collective the engines issued (captured or eager) must have completed before the
    communicator is freed: the device is synchronised first, and an engine built on it must not
    be stepped afterwards (its recorded Programs / graphs still name the freed ncclComm)."""
    global _PG_INITIALISED_HERE, _NATIVE
    if _NATIVE is not None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        _NATIVE.destroy()
        _NATIVE = None
    if is_initialized() and _PG_INITIALISED_HERE:
        dist.destroy_process_group()
        _PG_INITIALISED_HERE = False


def barrier() -> None:
    if is_initialized():
        dist.barrier()


def max_over_ranks(x: float, device: torch.device) -> float:
    if not is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_tensors(tensors: Sequence[torch.Tensor], src: int = 0) -> None:
    if not is_initialized():
        return
    for t in tensors:
        dist.broadcast(t, src=src)


def all_reduce_mean_(t: torch.Tensor) -> None:
    if not is_initialized():
        return
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t.mul_(1.0 / dist.get_world_size())


def any_rank(flag: bool, device: torch.device) -> bool:
    """Collective OR of a per-rank boolean (used to share the chief's save decision)."""
    if not is_initialized():
        return bool(flag)
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(int(t.item()))


def average_scalars(values: Sequence[float], device: torch.device) -> List[float]:
    """Mean of a few host scalars over ranks (logging steps only)."""
    if not is_initialized():
        return list(values)
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return (t / dist.get_world_size()).tolist()


def params_in_sync(tensors: Sequence[torch.Tensor], device: torch.device) -> bool:
    """Cross-rank divergence check: every rank hashes its parameters (exact
    bit pattern, order-sensitive), MIN and MAX of the hashes are all-reduced; equal <=> in sync."""
    if not is_initialized():
        return True
    h = torch.zeros(2, dtype=torch.int64, device=tensors[0].device)
    for i, t in enumerate(tensors):
        bits = t.detach().contiguous().view(torch.int32).to(torch.int64)
        w = torch.arange(1, bits.numel() + 1, device=bits.device, dtype=torch.int64) % 65521 + 1
        h[0] += ((bits * w).sum() * (i + 1)) & 0x3FFFFFFFFFFF
        h[1] += (bits.sum() * (2 * i + 3)) & 0x3FFFFFFFFFFF
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    lo = h.to(dev).clone()
    hi = h.to(dev).clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))


def make_buckets(numel: int, bucket_elems: int, align: int = 64) -> List[Tuple[int, int]]:
    """Split [0, numel) into contiguous (start, end) buckets of ~bucket_elems, 64-aligned."""
    bucket_elems = max(align, (bucket_elems // align) * align)
    out = []
    s = 0
    while s < numel:
        e = min(numel, s + bucket_elems)
        out.append((s, e))
        s = e
    return out


class GradAllReducer:
    """Bucketed, stream-overlapped all-reduce of one flat gradient buffer.

    ``launch()`` records an event on the compute stream, makes the comm stream wait on
    it and issues one all-reduce per bucket there (SUM); ``wait()`` makes the compute
    stream wait for the comm stream and applies the 1/W scale (folded into the Adam
    kernel on the HIP path via ``grad_scale``). With ``wire_dtype=bf16`` the buckets are
    converted to bf16 for the wire (half the xGMI bytes) and back to fp32 -- unless the caller
    hands in ``wire`` (a bf16 buffer it fills itself, e.g. from a cast kernel inside its step
    graph) with ``prefilled=True``: then only the wire is all-reduced, and the consumer (the HIP
    engine's Adam) reads the reduced bf16 values directly -- no copies around the collective.
    """

    def __init__(self, flat_grad: torch.Tensor, bucket_mb: float = 32.0, wire_dtype: str = "fp32",
                 reverse: bool = True, stream: "Optional[torch.cuda.Stream]" = None, force: bool = False,
                 wire: Optional[torch.Tensor] = None, prefilled: bool = False, native=None):
        self.flat = flat_grad
        self.native = native  # native_comm(): ncclAllReduce on the current stream, from C++
        self.world = world_size()
        # collectives are issued when there is a peer -- or on a forced one-rank group
        self.active = is_initialized() and (self.world > 1 or force)
        esize = 2 if wire_dtype == "bf16" else 4
        self.buckets = make_buckets(flat_grad.numel(), int(bucket_mb * 1024 * 1024 / esize))
        if reverse:  # gradients of the last layers are final first
            self.buckets = self.buckets[::-1]
        self.wire_dtype = wire_dtype
        # reducers of one engine share a comm stream: their collectives run in issue order
        self.stream = stream if stream is not None else (
            torch.cuda.Stream(device=flat_grad.device) if flat_grad.is_cuda else None)
        self.prefilled = bool(prefilled)
        if self.prefilled and (wire is None or wire_dtype != "bf16" or wire.numel() != flat_grad.numel()
                               or wire.dtype != torch.bfloat16):
            raise ValueError("prefilled needs a bf16 wire of the gradient's size")
        self.wire = (wire if wire is not None else
                     torch.empty(flat_grad.numel(), dtype=torch.bfloat16, device=flat_grad.device)
                     if wire_dtype == "bf16" else None)
        self._works = []

    def launch(self) -> None:
        if not self.active:
            return
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.flat.device)
            self.stream.wait_stream(cur)
            ctx = torch.cuda.stream(self.stream)
        else:
            ctx = _nullctx()
        with ctx:
            self.issue()

    def issue(self) -> None:
        """The bucket collectives on the CURRENT stream (the caller has ordered it after the
        producers of the gradients; the HIP engine's executor does this)."""
        if not self.active:
            return
        for s, e in self.buckets:
            if self.prefilled:
                self._sum(self.wire[s:e])
            elif self.wire is not None:
                w = self.wire[s:e]
                w.copy_(self.flat[s:e])
                self._sum(w)
                self.flat[s:e].copy_(w)
            else:
                self._sum(self.flat[s:e])

    def _sum(self, t: torch.Tensor) -> None:
        if self.native is not None:
            code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[t.dtype]
            self.native.all_reduce(t.data_ptr(), t.numel(), code, torch.cuda.current_stream(t.device).cuda_stream)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

    def accesses(self):
        """(ptr, bytes, is_write) ranges one issue() touches (schedule checker)."""
        out = [] if self.prefilled else [(self.flat.data_ptr(), self.flat.numel() * self.flat.element_size(), True)]
        if self.wire is not None:
            out.append((self.wire.data_ptr(), self.wire.numel() * self.wire.element_size(), True))
        return out

    def wait(self, scale_in_place: bool = True) -> None:
        if not self.active:
            return
        if self.stream is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
        if scale_in_place:
            if self.prefilled:
                self.flat.copy_(self.wire)
            self.flat.mul_(1.0 / self.world)


class ShardReducer:
    """One gradient slice of the sharded update (ZeRO-1 style): ``rs()``
    reduce-scatters the fp32 gradient slice (SUM) into this rank's shard ``gs`` (1/W of it); the
    caller's Adam updates that shard of the fp32 masters / slots and writes its 16-bit weights into
    ``agin``; ``ag()`` all-gathers ``agin`` from every rank into the mirror slice the GEMMs read.
    Per rank that is (W-1)/W x (4 + 2) bytes per element on the wire instead of the all-reduce's
    2 (W-1)/W x 4, at unchanged gradient precision, and 1/W of the Adam work. The slice length
    must be a multiple of W (ParamSet's 64-element alignment covers W | 64)."""

    def __init__(self, grad_slice: torch.Tensor, mirror_slice: torch.Tensor, world: Optional[int] = None,
                 rank_: Optional[int] = None):
        self.world = int(world or world_size())
        self.rank = rank() if rank_ is None else int(rank_)
        n = grad_slice.numel()
        if n % self.world or mirror_slice.numel() != n:
            raise ValueError("sharded slice of %d elements for %d ranks" % (n, self.world))
        self.grad, self.mirror = grad_slice, mirror_slice
        self.n = n // self.world
        self.lo = self.rank * self.n  # this rank's shard inside the slice
        self.gs = torch.empty(self.n, dtype=torch.float32, device=grad_slice.device)
        self.agin = torch.empty(self.n, dtype=mirror_slice.dtype, device=grad_slice.device)
        self.active = is_initialized()
        self.rs_op, self.ag_op = _ShardOp(self, True), _ShardOp(self, False)

    def rs(self) -> None:
        if self.active:
            dist.reduce_scatter_tensor(self.gs, self.grad, op=dist.ReduceOp.SUM)
        else:  # no process group (dry runs / one process): the shard is the slice itself
            self.gs.copy_(self.grad[self.lo:self.lo + self.n])

    def ag(self) -> None:
        if self.active:
            dist.all_gather_into_tensor(self.mirror, self.agin)
        else:
            self.mirror[self.lo:self.lo + self.n].copy_(self.agin)


class _ShardOp:
    """The reduce-scatter or the all-gather half of a ShardReducer, as an executor collective
    (``issue()`` on the current stream, ``accesses()`` for the schedule checker)."""

    def __init__(self, r: ShardReducer, is_rs: bool):
        self.r, self.is_rs = r, is_rs
        self.label = "%s[%d elems]" % ("reduce_scatter" if is_rs else "all_gather", r.grad.numel())

    def issue(self) -> None:
        self.r.rs() if self.is_rs else self.r.ag()

    def accesses(self):
        r = self.r
        if self.is_rs:
            return [(r.grad.data_ptr(), r.grad.numel() * 4, False), (r.gs.data_ptr(), r.n * 4, True)]
        es = r.mirror.element_size()
        return [(r.agin.data_ptr(), r.n * es, False), (r.mirror.data_ptr(), r.mirror.numel() * es, True)]


def gather_shards(flat: torch.Tensor, slices: Sequence[Tuple[int, int]]) -> None:
    """All-gather every rank's shard of each [a, b) slice of a flat fp32 buffer (masters / Adam
    slots after sharded updates) so that every rank holds the whole buffer again."""
    if not is_initialized():
        return
    W, r = dist.get_world_size(), dist.get_rank()
    for a, b in slices:
        n = (b - a) // W
        shard = flat[a + r * n:a + (r + 1) * n].clone()
        dist.all_gather_into_tensor(flat[a:b], shard)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

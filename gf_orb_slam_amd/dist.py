"""The config-5 start-up exchange over gf_dist_* (RCCL
over xGMI inside libgfslam), and the same protocol over a torch.distributed
process group (gloo) for CPU tests of the packing and the checksums.

Rank 0 builds the shared state — the rendered world (plane geometry and
textures of every scene), the ORB vocabulary and each stream's local map —
and broadcasts it; every rank then tracks its own sequences (its own phases
of the loops) with no further communication until the final timing
reduction. One process per GPU.
"""
from __future__ import annotations

import ctypes
import zlib

import numpy as np

from ._lib import check, lib


def checksum(a: np.ndarray) -> int:
    return zlib.crc32(np.ascontiguousarray(a).view(np.uint8).reshape(-1).tobytes()) & 0xFFFFFFFF


TRANSPORTS = {"rccl": 0, "loopback": 1, "host": 2}

# gf_dist_host_fn (abi.h): int fn(void* user, int op, void* host_buf, size_t bytes, int root)
HOST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)


class LoopbackChannel:
    """gf_dist_channel: the meeting point of `world` loopback ranks, each a
    host thread of this process with its own context (abi.h)."""

    def __init__(self, world: int):
        self.world = world
        self.handle = ctypes.c_void_p()
        check(lib().gf_dist_channel_create(world, ctypes.byref(self.handle)))

    def close(self) -> None:
        if self.handle:
            lib().gf_dist_channel_destroy(self.handle)
            self.handle = None


def _gloo_host_fn(pg):
    """The host-staged transport's collective over a torch.distributed group
    (gloo): broadcast of bytes from root, or an in-place all-reduce of
    doubles (abi.h GF_DIST_OP_*)."""
    import torch
    import torch.distributed as dist

    ops = {1: dist.ReduceOp.SUM, 2: dist.ReduceOp.MAX, 3: dist.ReduceOp.MIN}

    def fn(user, op, buf, nbytes, root):
        try:
            if nbytes == 0:
                return 0
            a = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(buf))
            if op == 0:
                dist.broadcast(torch.from_numpy(a), src=root, group=pg)
            else:
                dist.all_reduce(torch.from_numpy(a.view(np.float64)), op=ops[op], group=pg)
            return 0
        except Exception:  # noqa: BLE001 - reported to the library as a failed collective
            import traceback

            traceback.print_exc()
            return 1

    return HOST_FN(fn)


class GfDist:
    """A communicator of libgfslam (gf_dist_*) on one context's device.

    transport "rccl" (the product path): an RCCL communicator, the 128-byte
    unique id handed out over the torch.distributed group `pg`. "loopback":
    ranks are threads of this process meeting in `channel` (a LoopbackChannel)
    — one GPU runs the receiving side of every exchange. "host": host-staged
    collectives over the torch.distributed group `pg` (gloo), for processes
    sharing one GPU."""

    def __init__(self, ctx, rank: int, world: int, pg=None, transport: str = "rccl", channel=None):
        self.ctx, self.rank, self.world = ctx, rank, world
        self.transport = transport
        self.handle = ctypes.c_void_p()
        if transport == "loopback":
            if channel is None or channel.world != world:
                raise ValueError("loopback ranks need a LoopbackChannel of the same world size")
            self._channel = channel
            check(lib().gf_dist_init_loopback(ctx.handle, rank, channel.handle, ctypes.byref(self.handle)))
            return
        if transport == "host":
            self._fn = _gloo_host_fn(pg)  # kept alive for the communicator's lifetime
            check(lib().gf_dist_init_host(ctx.handle, rank, world, self._fn, None, ctypes.byref(self.handle)))
            return
        if transport != "rccl":
            raise ValueError(f"unknown transport {transport!r}")
        import torch
        import torch.distributed as dist

        uid = np.zeros(128, np.uint8)
        if rank == 0:
            check(lib().gf_dist_unique_id(uid.ctypes.data_as(ctypes.c_void_p)))
        if world > 1:
            t = torch.from_numpy(uid).to(f"cuda:{ctx.device}")
            dist.broadcast(t, src=0, group=pg)
            uid = t.cpu().numpy()
        check(lib().gf_dist_init(ctx.handle, rank, world, uid.ctypes.data_as(ctypes.c_void_p),
                                 ctypes.byref(self.handle)))

    def info(self) -> tuple[int, int]:
        """(rank, world) as the communicator holds them (gf_dist_info)."""
        r, w = ctypes.c_int(), ctypes.c_int()
        check(lib().gf_dist_info(self.handle, ctypes.byref(r), ctypes.byref(w)))
        return r.value, w.value

    def transport_kind(self) -> int:
        k = ctypes.c_int()
        check(lib().gf_dist_transport(self.handle, ctypes.byref(k)))
        return k.value

    def bcast_array(self, a: np.ndarray | None, root: int = 0) -> np.ndarray:
        """Broadcast a host byte array through a device buffer (size first)."""
        import torch

        dev = f"cuda:{self.ctx.device}"
        n = torch.tensor([float(a.nbytes) if self.rank == root else 0.0], dtype=torch.float64).to(dev)
        # the library broadcasts on its own (non-blocking) stream: torch's
        # stream must have finished writing the buffers before the call
        torch.cuda.current_stream(dev).synchronize()
        check(lib().gf_dist_bcast(self.handle, ctypes.c_void_p(n.data_ptr()), 8, root))
        nb = int(n.item())
        buf = torch.empty(nb, dtype=torch.uint8, device=dev)
        if self.rank == root:
            buf.copy_(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)))
        torch.cuda.current_stream(dev).synchronize()
        check(lib().gf_dist_bcast(self.handle, ctypes.c_void_p(buf.data_ptr()), nb, root))
        return buf.cpu().numpy()

    def bcast_vocab(self, voc, root: int = 0):
        from .bow import ORBVocabulary

        h = voc.handle if self.rank == root else ctypes.c_void_p()
        check(lib().gf_dist_bcast_vocab(self.handle, ctypes.byref(h), root))
        return voc if self.rank == root else ORBVocabulary.from_handle(h, self.ctx)

    def bcast_map(self, fe, root: int = 0) -> None:
        check(lib().gf_dist_bcast_map(self.handle, fe.handle, root))

    def gather_ints(self, vals) -> np.ndarray:
        """Every rank's values (max / min all-reduce pair): rows [min, max]."""
        import torch

        v = np.asarray(vals, np.float64)
        out = []
        for op in (2, 1):
            t = torch.from_numpy(v.copy()).to(f"cuda:{self.ctx.device}")
            torch.cuda.current_stream(t.device).synchronize()
            check(lib().gf_dist_allreduce(self.handle, ctypes.c_void_p(t.data_ptr()), len(v), op))
            out.append(t.cpu().numpy())
        return np.stack(out)

    def close(self) -> None:
        if self.handle:
            lib().gf_dist_destroy(self.handle)
            self.handle = None


class TorchComm:
    """The same byte broadcast over a torch.distributed group (gloo on CPU)."""

    def __init__(self, rank: int, world: int, pg=None):
        self.rank, self.world, self.pg = rank, world, pg

    def bcast_array(self, a: np.ndarray | None, root: int = 0) -> np.ndarray:
        import torch
        import torch.distributed as dist

        n = torch.zeros(1, dtype=torch.int64)
        if self.rank == root:
            n[0] = a.nbytes
        if self.world > 1:
            dist.broadcast(n, src=root, group=self.pg)
        buf = torch.zeros(int(n.item()), dtype=torch.uint8)
        if self.rank == root:
            buf.copy_(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)))
        if self.world > 1:
            dist.broadcast(buf, src=root, group=self.pg)
        return buf.numpy()

    def gather_ints(self, vals) -> np.ndarray:
        import torch
        import torch.distributed as dist

        v = torch.tensor(np.asarray(vals, np.float64))
        lo, hi = v.clone(), v.clone()
        if self.world > 1:
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.pg)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.pg)
        return np.stack([lo.numpy(), hi.numpy()])


# ------------------------------------------------------------- packing
def pack_world(scenes, maps) -> np.ndarray:
    """Scenes (Scene.pack) and per-scene maps in one blob: (points,
    descriptors), (points, descriptors, keyframe graph arrays) or with the
    keyframes' keypoints and descriptors too (the relocalisation database's
    inputs): (points, descriptors, graph, kf_kps, kf_desc)."""
    from .orb import KEYPOINT_DTYPE
    from .localmap import _ARRAYS
    from .matcher import MAP_POINT_DTYPE

    parts = []
    for sc, m in zip(scenes, maps):
        mp, d = m[0], m[1]
        g = m[2] if len(m) > 2 else None
        sb = sc.pack()
        mb = np.ascontiguousarray(mp, MAP_POINT_DTYPE).view(np.uint8).reshape(-1)
        db = np.ascontiguousarray(d, np.uint8).reshape(-1)
        kf = len(m) > 4
        if kf and g is None:  # the keyframe section is read only after a graph (header flag 2)
            raise ValueError("keyframe keypoints / descriptors need the keyframe graph (maps[2])")
        hdr = np.array([sb.nbytes, len(mp), 0 if g is None else (2 if kf else 1)], np.int64).view(np.uint8)
        parts += [hdr, sb, mb, db]
        if g is not None:
            for k, dt in _ARRAYS:
                a = np.ascontiguousarray(g[k], dt).reshape(-1)
                parts += [np.array([len(a)], np.int64).view(np.uint8), a.view(np.uint8)]
        if kf:
            parts.append(np.array([len(m[3])], np.int64).view(np.uint8))
            for kp, de in zip(m[3], m[4]):
                kp = np.ascontiguousarray(kp, KEYPOINT_DTYPE)
                parts += [np.array([len(kp)], np.int64).view(np.uint8), kp.view(np.uint8),
                          np.ascontiguousarray(de, np.uint8).reshape(-1)]
    return np.concatenate([np.array([len(scenes)], np.int64).view(np.uint8)] + parts)


def unpack_world(blob: np.ndarray):
    from .matcher import MAP_POINT_DTYPE
    from .scene import Scene

    from .localmap import _ARRAYS
    from .orb import KEYPOINT_DTYPE

    S = int(blob[:8].view(np.int64)[0])
    o = 8
    scenes, maps = [], []
    for _ in range(S):
        sb, m, hg = (int(x) for x in blob[o:o + 24].view(np.int64))
        o += 24
        scenes.append(Scene.unpack(blob[o:o + sb]))
        o += sb
        mp = blob[o:o + m * MAP_POINT_DTYPE.itemsize].copy().view(MAP_POINT_DTYPE)
        o += m * MAP_POINT_DTYPE.itemsize
        d = blob[o:o + 32 * m].copy().reshape(m, 32)
        o += 32 * m
        if hg:
            g = {}
            for k, dt in _ARRAYS:
                n = int(blob[o:o + 8].view(np.int64)[0])
                o += 8
                nb = n * np.dtype(dt).itemsize
                g[k] = blob[o:o + nb].copy().view(dt)
                o += nb
            if hg == 2:
                nkf = int(blob[o:o + 8].view(np.int64)[0])
                o += 8
                kps, des = [], []
                for _ in range(nkf):
                    n = int(blob[o:o + 8].view(np.int64)[0])
                    o += 8
                    kps.append(blob[o:o + n * KEYPOINT_DTYPE.itemsize].copy().view(KEYPOINT_DTYPE))
                    o += n * KEYPOINT_DTYPE.itemsize
                    des.append(blob[o:o + 32 * n].copy().reshape(n, 32))
                    o += 32 * n
                maps.append((mp, d, g, kps, des))
            else:
                maps.append((mp, d, g))
        else:
            maps.append((mp, d))
    return scenes, maps


def share_world(comm, rank: int, build) -> tuple:
    """Rank 0 calls build() -> (scenes, maps) and broadcasts them; returns
    (scenes, maps, blob checksum, [min, max] of every rank's checksum)."""
    blob = pack_world(*build()) if rank == 0 else None
    got = comm.bcast_array(blob, 0)
    ck = checksum(got)
    span = comm.gather_ints([ck])
    scenes, maps = unpack_world(got)
    return scenes, maps, ck, span, got.nbytes

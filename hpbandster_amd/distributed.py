"""Candidate sharding across GPUs (one process per GPU) with one exchange of the local winners.

The reference's acquisition loop (bohb.py:133-152) scores candidates independently, so each rank
scores its contiguous shard with global indices (``index_base``) and runs the exact acquisition on it
(``KDEPair.acquire``).  The global winner is the minimum over ranks of (score, global index): one
collective, ``hbx_argmax_allreduce`` -- an RCCL all-gather over xGMI of every rank's 48-byte result
record, reduced on the device (libhbx's own RCCL communicator, no torch.distributed on the data path).
Ties across shards go to the smaller index, which preserves the reference's strict '<' first-index
rule.  A ``records`` transport does the same over ``torch.distributed`` (gloo on CPU, for rehearsals
of the multi-process path on one GPU, where RCCL refuses two ranks per device).

Exactness across ranks: every rank's exact score is the reference's float64 value bit for bit, so the
(score, index) reduction is the reference's pick.  With ties='process' (see KDEPair.acquire), winners
of different ranks within each other's numpy-build spread (``HBX_ACQ_NEAR_TIE``) are re-scored with
this process's numpy (``exact_host``) and a second exchange of those scores decides.
"""

import struct

import numpy as np

from . import _native as N

REC_BYTES = 48  # AcqResult (include/hbx.h)


def shard_range(n_total, rank, world):
    """Contiguous [lo, hi) of rank's candidates (sizes differ by at most one)."""
    q, r = divmod(int(n_total), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _unpack(raw):
    from .kde import AcqResult
    return AcqResult.from_bytes(raw)


def reduce_records_host(recs):
    """Host restatement of hbx_dist.hip's reduction over per-rank AcqResult records:
    (best rank or -1, ranks whose winners lie within the bounds of the best one)."""
    best = -1
    for r, a in enumerate(recs):
        if a.index < 0 or not a.score < np.inf:
            continue
        if best < 0 or a.score < recs[best].score or (a.score == recs[best].score and a.index < recs[best].index):
            best = r
    if best < 0:
        return -1, []
    b = recs[best]
    near = [r for r, a in enumerate(recs) if a.index >= 0 and a.score < np.inf and
            (r == best or a.score <= b.score * (1.0 + 1.0001 * (a.rel + b.rel)))]
    return best, near


def reduce_winners(score, index, group=None, device=None, rel=0.0):
    """All ranks' (score, index) -> global (index, score) over torch.distributed (any backend); index -1
    when no rank has a finite score.  ``score``: the exact score of the local winner."""
    import torch
    import torch.distributed as dist
    from .kde import AcqResult, RESULT_FMT
    ok = index >= 0 and np.isfinite(score)
    raw = struct.pack(RESULT_FMT, int(index) if ok else -1, float(score) if ok else np.nan, float(rel), 0, 0, 1,
                      np.nan, np.nan)
    loc = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    if device is not None:
        loc = loc.to(device)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world > 1:
        parts = [torch.empty_like(loc) for _ in range(world)]
        dist.all_gather(parts, loc, group=group)
        allr = [p.cpu().numpy().tobytes() for p in parts]
    else:
        allr = [loc.cpu().numpy().tobytes()]
    recs = [AcqResult.from_bytes(b) for b in allr]
    best, _ = reduce_records_host(recs)
    if best < 0:
        return -1, np.nan
    return recs[best].index, float(recs[best].score)


def broadcast_from_group_root(payload, group, world):
    """``payload`` of the group's rank 0 on every rank of ``group``.  broadcast_object_list takes a
    GLOBAL source rank: the group's rank 0 is global rank get_global_rank(group, 0), which is 0 only for
    the default group."""
    import torch.distributed as dist
    if world <= 1:
        return payload
    src = dist.get_global_rank(group, 0) if group is not None else 0
    box = [payload]
    dist.broadcast_object_list(box, src=src, group=group)
    return box[0]


class WinnerExchange(object):
    """The per-acquisition collective of a candidate-sharded run.

    ``transport='rccl'``: libhbx's own RCCL communicator (its unique id travels once through
    torch.distributed's default group at construction), ``hbx_argmax_allreduce`` on the device.
    ``transport='records'``: torch.distributed all_gather of the records through host memory (e.g. gloo),
    then the same device reduction (``hbx_argmax_records``).
    ``transport='torch'``: the same all_gather of the device records on torch's own process group (its
    nccl backend is RCCL as well) -- the fallback when libhbx's communicator cannot be set up.
    """

    def __init__(self, device, transport="rccl", group=None):
        import torch
        import torch.distributed as dist
        self.device = device
        self.group = group
        self.transport = transport
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        L = N.lib()
        with N.on_device(device):
            self.gather = torch.empty(int(L.hbx_argmax_gather_bytes(self.world)), dtype=torch.uint8, device=device)
            self.out = torch.empty(REC_BYTES, dtype=torch.uint8, device=device)
        self.comm = None
        if transport == "rccl":
            uid = bytearray(int(L.hbx_rccl_unique_id_bytes()))
            if self.rank == 0:
                buf = (np.frombuffer(uid, dtype=np.uint8)).copy()
                N.check(L.hbx_rccl_get_unique_id(N.ptr(buf)))
                uid = bytearray(buf.tobytes())
            uid = broadcast_from_group_root(bytes(uid), group, self.world)
            import ctypes
            idb = np.frombuffer(bytes(uid), dtype=np.uint8).copy()
            h = ctypes.c_void_p()
            dev = torch.device(device)
            dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
            # hbx_rccl_comm_init selects the device itself: inside on_device, torch's current device is
            # restored afterwards
            with N.on_device(torch.device("cuda", dev_index)):
                N.check(L.hbx_rccl_comm_init(ctypes.addressof(h), self.world, N.ptr(idb), self.rank, dev_index))
            self.comm = h.value
        elif transport not in ("records", "torch"):
            raise ValueError("transport must be 'rccl', 'records' or 'torch'")

    def exchange(self, rec, stream=None):
        """rec: this rank's device record (48 uint8) -> the global winner's device record (self.out);
        self.gather then holds every rank's record."""
        import torch
        import torch.distributed as dist
        L = N.lib()
        with N.on_device(self.device, stream):
            sh = N.stream_handle(stream, self.device)
            if self.transport == "rccl":
                N.check(L.hbx_argmax_allreduce(N.ptr(rec), N.ptr(self.gather), N.ptr(self.out), self.world, self.comm,
                                               sh))
            else:
                if self.world > 1:
                    loc = rec.cpu() if self.transport == "records" else rec[:REC_BYTES]
                    parts = [torch.empty_like(loc) for _ in range(self.world)]
                    dist.all_gather(parts, loc, group=self.group)
                    self.gather.copy_(torch.cat(parts))
                else:
                    self.gather.copy_(rec)
                N.check(L.hbx_argmax_records(N.ptr(self.gather), self.world, N.ptr(self.out), sh))
        return self.out

    def rccl_world_size(self):
        """The rank count of libhbx's communicator as RCCL reports it (ncclCommCount); None for the
        records transport."""
        if self.comm is None:
            return None
        import ctypes
        c = ctypes.c_int32(0)
        N.check(N.lib().hbx_rccl_comm_count(self.comm, ctypes.addressof(c)))
        return int(c.value)

    def records(self):
        raw = self.gather.cpu().numpy().tobytes()
        return [_unpack(raw[r * REC_BYTES:(r + 1) * REC_BYTES]) for r in range(self.world)]

    def close(self):
        if self.comm is not None:
            N.lib().hbx_rccl_comm_destroy(self.comm)
            self.comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def acquire_sharded(pair, cands_local, index_base, exchange, stream=None, workspace=None, ties="pinned",
                    events=None):
    """Exact acquisition on this rank's shard, then the global winner: (index, score, AcqResult).

    One collective.  With ties='process' (KDEPair.acquire), a near tie across ranks adds a host
    re-score of the ranks' near sets in this process's numpy and a second exchange of those scores."""
    import torch
    from . import exact_host
    from .kde import AcqResult, RESULT_FMT, ACQ_NEAR_TIE, ACQ_RESOLVED, _rows_of, fetch_bytes
    Nc = int(cands_local.shape[0])
    with N.on_device(pair.good.device, stream):
        ws = workspace if workspace is not None else torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8,
                                                                 device=pair.good.device)
        rv = pair.acquire(cands_local, index_base=index_base, stream=stream, workspace=ws, sync=False,
                          events=events)
        g = _unpack(fetch_bytes(exchange.exchange(rv, stream), stream))
        if ties != "process" or not g.flags & ACQ_NEAR_TIE:
            return g.index, g.score, g
        recs = exchange.records()
        best, near = reduce_records_host(recs)
        mine = _unpack(fetch_bytes(rv, stream))
        pick = None
        if exchange.rank in near:
            # every candidate of this rank's shortlist (indices local to the shard): its own near set is
            # taken against its own winner's bound, and for signed KDEs (per-candidate rel) a candidate can
            # lie within the GLOBAL winner's bound yet outside its rank winner's -- the shortlist holds both
            o = pair._ws_offsets(Nc, Nc)
            cnt = int(ws[o[0]:o[0] + 4].view(torch.int32).item())
            idx = np.unique(ws[o[1]:o[1] + 4 * cnt].view(torch.int32).cpu().numpy().astype(np.int64))
            if idx.size == 0:
                idx = np.array([mine.index - index_base], dtype=np.int64)
            pick = exact_host.resolve(pair.good, pair.bad, _rows_of(cands_local, idx), idx)
        if pick is None:
            raw = struct.pack(RESULT_FMT, -1, np.nan, 0.0, 0, 0, 0, np.nan, np.nan)
        else:
            raw = struct.pack(RESULT_FMT, pick[0] + index_base, pick[1], 0.0, ACQ_RESOLVED, 0, 1, pick[2], pick[3])
        rec = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(pair.good.device)
        g2 = _unpack(fetch_bytes(exchange.exchange(rec, stream), stream))
        g2.flags |= ACQ_RESOLVED
        return g2.index, g2.score, g2

"""Multi-GPU sharding of the hot path (one process per GPU, torch.distributed).

trackingCT.m's channels are independent (the `for svindex` loop re-initialises
everything, trackingCT.m:22-528) and acquisition.m's PRNs too
(acquisition.m:47-80), so the path shards with no per-step communication:

  * acquisition: PRNs round-robin over ranks; each rank searches its PRNs on its
    GPU; one all-gather of the fixed-size per-PRN records assembles the
    reference's ascending-PRN Acquired struct on every rank;
  * trackingCT: channels round-robin over ranks (the GLOBAL svindex/nsv are kept
    for the linear-indexing quirk of trackingCT.m:161); per-channel series are
    gathered to rank 0 (or all ranks) at the end.

The collective backend is whatever the process group uses: "nccl" (= RCCL over
xGMI on MI355X) on the GPU box, "gloo" for the CPU tests.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np


def shard(n: int, world: int, rank: int) -> list[int]:
    """Round-robin indices of `n` units owned by `rank`."""
    return list(range(rank, n, world))


def _all_gather_array(arr: np.ndarray, group=None, device=None) -> list[np.ndarray]:
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [o.cpu().numpy() for o in out]


def gather_acquired(local, prns_local, world_prns, group=None, device=None):
    """Merge per-rank Acquired structs into the reference's ascending-PRN struct.

    local: Acquired of this rank's PRNs (sv, SNR, Doppler, codedelay, fineFreq).
    Each rank packs a fixed-size record table (one row per PRN of the whole search,
    NaN where not acquired here) and one all-gather merges them.
    """
    allp = sorted(world_prns)
    tab = np.full((len(allp), 5), np.nan)
    pos = {p: i for i, p in enumerate(allp)}
    for k, sv in enumerate(local.sv):
        tab[pos[int(sv)]] = [sv, local.SNR[k], local.Doppler[k], local.codedelay[k], local.fineFreq[k]]
    parts = _all_gather_array(tab, group, device)
    merged = np.full_like(tab, np.nan)
    for t in parts:
        have = ~np.isnan(t[:, 0])
        merged[have] = t[have]
    rows = merged[~np.isnan(merged[:, 0])]
    return SimpleNamespace(sv=rows[:, 0].astype(np.int64), SNR=rows[:, 1], Doppler=rows[:, 2],
                           codedelay=rows[:, 3].astype(np.int64), fineFreq=rows[:, 4])


def gather_tracking_rows(buf, shards, group=None, device=None):
    """All-gather only the channel rows each rank tracked (rank r owns shards[r], e.g.
    shard(nsv, world, r)): every rank sends its own rows of rec / len / countinx / CN0
    columns (padded to the largest shard) and writes the others' rows into `buf`, which
    then holds the full result on every rank. Traffic per rank = its own rows, not the
    whole buffer."""
    import torch.distributed as dist
    me = dist.get_rank(group)
    width = max(len(s) for s in shards)
    mine = list(shards[me])
    rec = np.zeros((width,) + buf.rec.shape[1:], dtype=buf.rec.dtype)
    rec[: len(mine)] = buf.rec[mine]
    meta = np.zeros((width, 2), dtype=np.int64)
    meta[: len(mine), 0] = buf.len[mine]
    meta[: len(mine), 1] = buf.countinx[mine]
    cn0 = np.zeros((buf.CN0.shape[0], width))
    cn0[:, : len(mine)] = buf.CN0[:, mine]
    rows = np.array([buf.c.cn0_rows], dtype=np.int64)
    parts = zip(_all_gather_array(rec, group, device), _all_gather_array(meta, group, device),
                _all_gather_array(cn0, group, device))
    for r, (pr, pm, pc) in enumerate(parts):
        if r == me:
            continue
        ch = list(shards[r])
        buf.rec[ch] = pr[: len(ch)]
        buf.len[ch] = pm[: len(ch), 0]
        buf.countinx[ch] = pm[: len(ch), 1]
        buf.CN0[:, ch] = pc[:, : len(ch)]
    if buf.taps is not None:  # the ACF taps (config 5): the largest per-channel payload
        taps = np.zeros((width,) + buf.taps.shape[1:], dtype=buf.taps.dtype)
        taps[: len(mine)] = buf.taps[mine]
        for r, pt in enumerate(_all_gather_array(taps, group, device)):
            if r != me:
                buf.taps[list(shards[r])] = pt[: len(shards[r])]
    buf.c.cn0_rows = int(max(_all_gather_array(rows, group, device))[0])
    return buf


def _gather_into(out, t, group):
    """all_gather_into_tensor; gloo with device tensors (the one-GPU rehearsal) takes the
    list form."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), t, group=group)
    else:
        dist.all_gather_into_tensor(out, t, group=group)


def gather_tracking_rows_device(buf, shards, group=None, defer=False):
    """gather_tracking_rows for DeviceTrackOutBuffers: the TckResultCT series (rec, and
    taps when present) never leave HBM -- each rank packs its own channels' rows on the GPU
    and one all_gather_into_tensor (RCCL over xGMI on MI355X) delivers every rank's rows,
    scattered back in place. The small host arrays (len, countinx, CN0 columns, cn0_rows)
    travel in one packed device tensor of their own.

    defer=True: enqueue the device work and return a function that completes the gather
    (the one host round trip: the packed metadata's copy back and its scatter into the host
    arrays), so the caller can start other GPU work first. Call it before anything writes or
    reads `buf` again."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    width = max(len(s) for s in shards)
    dev = buf.rec.device
    mine = torch.tensor(list(shards[me]), dtype=torch.long, device=dev)

    def rows(t):
        own = torch.zeros((width,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        own[: len(shards[me])] = t.index_select(0, mine)
        allr = torch.empty((world * width,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        _gather_into(allr, own, group)
        for r in range(world):
            if r != me and len(shards[r]):
                idx = torch.tensor(list(shards[r]), dtype=torch.long, device=dev)
                t.index_copy_(0, idx, allr[r * width: r * width + len(shards[r])])

    rows(buf.rec)
    if buf.taps is not None:
        rows(buf.taps)
    # small per-channel metadata: [len, countinx, CN0 column ...] per owned channel
    nc = buf.CN0.shape[0]
    meta = np.zeros((width, 3 + nc))
    for j, c in enumerate(shards[me]):
        meta[j, 0], meta[j, 1], meta[j, 2] = buf.len[c], buf.countinx[c], buf.c.cn0_rows
        meta[j, 3:] = buf.CN0[:, c]
    mt = torch.from_numpy(meta).to(dev, non_blocking=False)
    allm_d = torch.empty((world * width, 3 + nc), dtype=mt.dtype, device=dev)
    _gather_into(allm_d, mt, group)

    def finish():
        allm = allm_d.cpu().numpy()
        crows = buf.c.cn0_rows
        for r in range(world):
            for j, c in enumerate(shards[r]):
                m = allm[r * width + j]
                crows = max(crows, int(m[2]))
                if r != me:
                    buf.len[c], buf.countinx[c] = int(m[0]), int(m[1])
                    buf.CN0[:, c] = m[3:]
        buf.c.cn0_rows = crows
        return buf

    return finish if defer else finish()


def gather_tracking(buf, nsv: int, group=None, device=None):
    """All-gather the channel rows each rank filled in its TrackOutBuffers.

    Every rank owns disjoint channels (rows of rec / taps / len / countinx /
    CN0 columns); rows a rank did not track are zero there, so the element-wise
    sum of the gathered buffers is the full result.
    """
    rec = sum(_all_gather_array(buf.rec, group, device))
    length = sum(_all_gather_array(buf.len, group, device))
    cx = sum(_all_gather_array(buf.countinx.astype(np.int64), group, device))
    cn0 = sum(_all_gather_array(buf.CN0, group, device))
    taps = sum(_all_gather_array(buf.taps, group, device)) if buf.taps is not None else None
    rows = int(max(_all_gather_array(np.array([buf.c.cn0_rows]), group, device))[0])
    return SimpleNamespace(rec=rec, len=length, countinx=cx, CN0=cn0[:rows], taps=taps,
                           cn0_rows=rows)

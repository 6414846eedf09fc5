"""Cross-GPU stripe placement.

When a storage layer spreads the shards of one stripe over several GPUs (one
process per GPU), rebuilding a lost shard needs d survivors that live on
other GPUs.  `gather_reconst` moves exactly those survivors to each stripe's
owner with one all-to-all (RCCL over xGMI with the "nccl" backend; gloo on
CPU for tests), decodes every owned stripe in one multi-pattern launch
(rs_reconst_batch_multi) and, optionally, sends each rebuilt shard back to
its home rank with a second all-to-all.

Survivor choice follows the reference: the first d surviving vectors in
index order (rs.go:264-330 checkReconst), so the decode is
byte-identical to a single-GPU Reconst of the same stripe.

Placement is rotating by default — shard v of stripe s lives on rank
(s + v) % world and stripe s is decoded on rank s % world — and can be
replaced by any pair of functions every rank agrees on.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .rs import ErrIllegalVects, ErrInvalidArgument, ErrTooManyLost

Shard = Tuple[int, int]  # (stripe, vector)


class Placement:
    """Where every shard lives and where every stripe is decoded."""

    def __init__(self, data_num: int, parity_num: int, world: int, nstripes: int,
                 home: Optional[Callable[[int, int], int]] = None,
                 owner: Optional[Callable[[int], int]] = None):
        if world <= 0 or nstripes < 0:
            raise ErrInvalidArgument()
        self.d, self.p, self.world, self.nstripes = data_num, parity_num, world, nstripes
        self.home = home or (lambda s, v: (s + v) % world)
        self.owner = owner or (lambda s: s % world)

    def local_shards(self, rank: int) -> List[Shard]:
        """The shards rank holds, in the order of its local tensor's rows."""
        n = self.d + self.p
        return [(s, v) for s in range(self.nstripes) for v in range(n) if self.home(s, v) == rank]

    def local_index(self, rank: int) -> Dict[Shard, int]:
        return {sv: i for i, sv in enumerate(self.local_shards(rank))}


def _plan(pl: Placement, need_masks: np.ndarray):
    """Per stripe with erasures: the d survivors used (index order) and the lost set."""
    n = pl.d + pl.p
    valid = (1 << n) - 1
    plan = {}
    for s in range(pl.nstripes):
        m = int(need_masks[s])
        if not m:
            continue
        if m & ~valid:
            raise ErrIllegalVects()
        lost = [v for v in range(n) if m >> v & 1]
        if len(lost) > pl.p:
            raise ErrTooManyLost()
        surv = [v for v in range(n) if not m >> v & 1][:pl.d]
        plan[s] = (surv, lost)
    return plan


def _all_to_all(dist, group, send, send_counts, recv_counts, vec, device, comm_device):
    """Rows of `send` (grouped by destination rank) -> rows from every source."""
    import torch

    send = send.reshape(-1).to(comm_device)
    recv = torch.empty(sum(recv_counts) * vec, dtype=torch.uint8, device=comm_device)
    dist.all_to_all_single(recv, send, [c * vec for c in recv_counts], [c * vec for c in send_counts], group=group)
    return recv.reshape(-1, vec).to(device)


def gather_reconst(codec, local, placement: Placement, need_masks: Sequence[int], rank: int,
                   group=None, write_back: bool = True,
                   decode: Optional[Callable] = None) -> Dict[Shard, "object"]:
    """Rebuild every shard marked in need_masks (need_masks[s] = bitmap of the
    lost vectors of stripe s, identical on every rank).

    local: this rank's shards, a [len(placement.local_shards(rank)), vec]
    uint8 tensor (lost rows hold garbage).  Returns {(s, v): row} for the
    shards rebuilt on this rank (the stripes it owns); with write_back every
    rebuilt shard is also copied into its home rank's `local` row.

    decode(work, masks): defaults to codec.reconst_batch_multi over the
    owned stripes' [S, d+p, vec] buffer; tests on CPU pass a stand-in.
    Every gather / scatter of rows is one indexed copy (no per-shard launches).
    """
    import torch
    import torch.distributed as dist

    pl = placement
    n, world, vec = pl.d + pl.p, pl.world, int(local.shape[1])
    masks = np.ascontiguousarray(np.asarray(need_masks, dtype=np.uint64))
    if masks.shape != (pl.nstripes,) or local.shape[0] != len(pl.local_shards(rank)):
        raise ErrInvalidArgument()
    plan = _plan(pl, masks)  # validates on every rank before any communication
    device = local.device
    comm_device = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    lidx = pl.local_index(rank)
    owned = [s for s in sorted(plan) if pl.owner(s) == rank]
    slot = {s: i for i, s in enumerate(owned)}
    ix = lambda xs: torch.tensor(xs, dtype=torch.long, device=device)  # noqa: E731

    # 1) survivors -> owners; canonical order (stripe, vector) inside each block
    send_rows = [[] for _ in range(world)]   # local rows, per destination
    recv_dest = [[] for _ in range(world)]   # work rows, per source
    for s, (surv, _lost) in sorted(plan.items()):
        o = pl.owner(s)
        for v in surv:
            h = pl.home(s, v)
            if h == rank:
                send_rows[o].append(lidx[(s, v)])
            if o == rank:
                recv_dest[h].append(slot[s] * n + v)
    flat = [r for dst in send_rows for r in dst]
    got = _all_to_all(dist, group, local.index_select(0, ix(flat)), [len(x) for x in send_rows],
                      [len(x) for x in recv_dest], vec, device, comm_device)

    # 2) decode the owned stripes in one launch
    rebuilt: Dict[Shard, object] = {}
    work = torch.zeros((len(owned), n, vec), dtype=torch.uint8, device=device)
    if owned:
        work.view(-1, vec).index_copy_(0, ix([r for src in recv_dest for r in src]), got)
        m_own = masks[owned]
        if decode is None:
            codec.reconst_batch_multi(work[:, :pl.d], work[:, pl.d:], m_own)
        else:
            decode(work, m_own)
        for s in owned:
            for v in plan[s][1]:
                rebuilt[(s, v)] = work[slot[s], v]

    # 3) rebuilt shards -> their homes
    if write_back:
        send_rows = [[] for _ in range(world)]  # work rows, per destination
        recv_dest = [[] for _ in range(world)]  # local rows, per source
        for s, (_surv, lost) in sorted(plan.items()):
            o = pl.owner(s)
            for v in lost:
                h = pl.home(s, v)
                if o == rank:
                    send_rows[h].append(slot[s] * n + v)
                if h == rank:
                    recv_dest[o].append(lidx[(s, v)])
        flat = [r for dst in send_rows for r in dst]
        back = _all_to_all(dist, group, work.view(-1, vec).index_select(0, ix(flat)), [len(x) for x in send_rows],
                           [len(x) for x in recv_dest], vec, device, comm_device)
        dest = [r for src in recv_dest for r in src]
        if dest:
            local.index_copy_(0, ix(dest), back)
    return rebuilt

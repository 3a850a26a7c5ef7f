"""The block-Hungarian round loop — my_optimizer of mpi_single.py:110-182 and
mpi_twins.py:112-188, one process per GPU.

Per round:
  sample disjoint blocks (A1) -> every rank solves its shard of the blocks
  on its GPU, fused cost build + LSAP + apply (A2-A6) -> ranks re-synchronise
  the gift-type vector with one all-gather (the reference's send/recv +
  bcast, mpi_single.py:136-152) -> every rank re-scores (A7, :157) ->
  accept / patience (A8, :160-169).

Semantics kept from the reference:
  * singles (accept="always"): the new state is always kept — subm_best is
    an alias of subm at mpi_single.py:113 and current_gift_ids is never
    reverted — and the loop stops after `patience`+1 consecutive rounds
    without a new best score (count > 3);
  * twins (accept="improve"): a round is kept only if the score improves,
    otherwise rolled back (mpi_twins.py:133,166-175); same stop rule;
  * triplets (an extension, accept="improve" as twins): 3-slot units, which
    the reference only asserts (mpi_single.py:32-37).
Pipelined round (an engine with score_begin): round r's score is computed
from a snapshot on a side stream while round r+1 is sampled and solved from
round r's result; the decisions of round r are taken one round late: if the
stop rule fires, round r+1's speculative update is undone; if round r is
rejected (keep-if-improved), the state returns to round r's starting
snapshot and round r+1 is run again from it.  Results and history equal the
serial loop's.
The reference uses `size` blocks per round (one per MPI rank); the default
here is every disjoint block of the round ("full"), and
`blocks_per_round=size` reproduces the reference's schedule.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib


@dataclass
class World:
    rank: int = 0
    size: int = 1
    group: object = None

    @property
    def distributed(self) -> bool:
        return self.size > 1


def shard_range(B: int, rank: int, size: int) -> tuple[int, int, int]:
    """Blocks [b0, b1) of rank `rank`; every rank gets `per` slots (padded)."""
    per = (B + size - 1) // size
    b0 = min(B, rank * per)
    b1 = min(B, b0 + per)
    return b0, b1, per


def all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """Rank-ordered concatenation of every rank's `inp` into `out` (RCCL
    all-gather over xGMI on GPUs).  An all-gather only moves bytes, and
    neither torch's NCCL/RCCL process group nor gloo maps int16, so int16
    buffers travel as their uint8 bytes (no copy, same HBM bytes).
    async_op: return the work handle (wait() before reading `out`)."""
    import torch.distributed as dist
    if inp.dtype == torch.int16:
        inp, out = inp.contiguous().view(torch.uint8), out.view(torch.uint8)
    try:
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    except (RuntimeError, AttributeError, NotImplementedError):
        parts = list(out.chunk(dist.get_world_size(group)))
        return dist.all_gather(parts, inp, group=group, async_op=async_op)


@dataclass
class RoundStats:
    round: int
    s_child: int
    s_gift: int
    score: float
    accepted: bool
    best: float
    blocks: int
    seconds: float


@dataclass
class LoopResult:
    history: list = field(default_factory=list)
    best_score: float = float("-inf")
    rounds: int = 0
    blocks_solved: int = 0
    sums: tuple | None = None  # exact (S_child, S_gift) of the final state


def exchange(engine, world: World, mode: int, rows: torch.Tensor, n: int, B: int,
             types: torch.Tensor, buffers: dict, during=None) -> None:
    """Make every rank's type vector identical after each solved its shard.

    Each rank packs the new types of its own blocks' rows (first twin only
    for pairs), one all-gather concatenates the shards in rank order (each
    padded to `per` blocks), and every rank scatters all of them.  Rank r's
    slice starts at r*per*n, which is where its blocks start in `rows`, and
    only trailing slots are padding, so recv[:B*n] lines up with rows[:B*n].
    during: work enqueued on the round's stream while the all-gather runs
    (it must not touch `types`; the round loop samples the next round's
    blocks there), before the unpack waits for the collective."""
    b0, b1, per = shard_range(B, world.rank, world.size)
    cnt = per * n
    key = (cnt, world.size)
    if buffers.get("key") != key:
        dev = types.device
        buffers["key"] = key
        buffers["send"] = torch.full((cnt,), -1, dtype=torch.int16, device=dev)
        buffers["recv"] = torch.empty((cnt * world.size,), dtype=torch.int16, device=dev)
    send, recv = buffers["send"], buffers["recv"]
    mine = rows[b0 * n:b1 * n]
    if mine.numel():
        engine.pack_types(types, mine, send[:mine.numel()])
    if during is None:
        all_gather_flat(recv, send, world.group)
    else:
        work = all_gather_flat(recv, send, world.group, async_op=True)
        during()
        work.wait()
    engine.unpack_types(types, rows[:B * n], recv[:B * n], mode)


ERROR_FLAG_BITS = 8  # SH_ERRF_* bits agreed across ranks (include/santa_hip.h)


def check_engine_errors(engine, world: World | None = None, device=None) -> None:
    """Raise if the device flagged a skipped block since the last check (an
    out-of-range child id or gift type, an infeasible solve: the kernels
    leave such a block's types unchanged, which would otherwise be scored
    and accepted silently).  Synchronises the engine's stream.

    With several ranks every rank must call this at the same point: the
    flags are agreed first (one all-reduce(MAX) of one int per flag bit:
    NCCL/RCCL has no bitwise-or reduction), so either every rank raises or
    none does -- a rank raising alone would leave the others waiting in the
    next collective."""
    read = getattr(engine, "error_flags", None)
    flags = read() if read is not None else 0
    if world is not None and world.distributed:
        import torch.distributed as dist
        bits = torch.tensor([(flags >> i) & 1 for i in range(ERROR_FLAG_BITS)], dtype=torch.int64,
                            device=device)
        dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=world.group)
        flags = sum(int(b) << i for i, b in enumerate(bits.tolist()))
    if flags:
        raise RuntimeError(f"sh_solve_blocks skipped blocks (device error flags {flags:#x}: "
                           f"{_lib.describe_error_flags(flags)})")


class _Sums:
    """Where a round's (S_child, S_gift) come from.

    full (check_every == 0): a rescore of the whole state every round, as the
    reference does on every rank (mpi_single.py:157).
    delta (check_every = K > 0; the default, K = 16): every
    rank's block kernels add the exact happiness deltas of ITS blocks into an
    int64[2], one all-reduce(sum) of those 16 bytes (RCCL over xGMI; the
    identity on one rank) gives the round's delta, and S = S(start state of
    the round) + delta; a full rescore of the state every K rounds (and after
    the last round) must agree, or the run stops with an error.  Integer
    sums: order-free, bit-exact -- every round's score equals the full
    rescore's, at every N (round 3: one GPU also takes its sums from the
    deltas, 2.5 % per round: profiles/r03_score_mode_ab.jsonl)."""

    def __init__(self, engine, world: World, check_every: int | None, max_rounds: int):
        if check_every is None:
            check_every = 16
        self.every = int(check_every) if hasattr(engine, "delta_begin") else 0
        self.engine, self.world, self.max_rounds = engine, world, max_rounds
        self.bufs = [engine.new_delta() for _ in range(2)] if self.every else None

    @property
    def delta(self) -> bool:
        return self.every > 0

    def check_round(self, rnd: int) -> bool:
        return (rnd + 1) % self.every == 0 or rnd == self.max_rounds - 1

    def buffer(self, k: int):
        d = self.bufs[k]
        zeroed = getattr(self.engine, "zeroed_delta", None)
        if zeroed is not None:  # (GPUEngine: zeroed ahead of time, off the round's stream)
            return zeroed(d)
        d.zero_()
        return d

    def reduce(self, d):
        """Start the all-reduce(sum) of d; returns its work handle (None on one
        rank).  The round's stream does not wait for it: the engine's
        delta_begin(after=work) makes the reader of d (the side stream) wait,
        so the 16-byte collective overlaps the next round's solve."""
        if self.world.distributed:
            import torch.distributed as dist
            return dist.all_reduce(d, group=self.world.group, async_op=True)
        return None

    @staticmethod
    def combine(base, rnd, dc, dg, full):
        """(S_child, S_gift, bad_triplets, bad_twins) of the round's state from
        the start state's sums and the all-reduced delta (checked against the
        full rescore when one was taken)."""
        sc, sg = base[0] + dc, base[1] + dg
        if full is None:
            return sc, sg, 0, 0
        if (full[0], full[1]) != (sc, sg):
            raise RuntimeError(f"round {rnd}: delta sums ({sc}, {sg}) != full rescore ({full[0]}, {full[1]})")
        return full

    def final_check(self, types, cur, history) -> None:
        """The loop ended (round budget or patience stop): unless the last
        round was a kept check round, its full rescore having confirmed `cur`,
        rescore the final state once; it must equal `cur`, and the family
        checks (mpi_single.py:32-44), which delta rounds skip, must pass."""
        if not self.delta or not history:
            return
        last = history[-1]
        if last.accepted and self.check_round(last.round):
            return
        full = tuple(self.engine.score_sums(types))
        if (full[0], full[1]) != tuple(cur):
            raise RuntimeError(f"final state: delta sums ({cur[0]}, {cur[1]}) != full rescore "
                               f"({full[0]}, {full[1]})")
        if full[2] or full[3]:
            raise AssertionError("triplets/twins must share a gift (mpi_single.py:32-44)")


def run_rounds(engine, types: torch.Tensor, *, mode: int = _lib.SH_MODE_SINGLE, n: int = 256,
               blocks_per_round: int | None = None, seed: int = 2017, max_rounds: int = 100,
               accept: str | None = None, patience: int = 3, world: World | None = None,
               on_round=None, score0: float | None = None, sums0: tuple | None = None,
               check_disjoint: bool = False, pipeline: bool = False,
               score_check_every: int | None = None) -> LoopResult:
    """The reference's while-loop; `types` (device int16 [nc]) is updated in place.

    accept: "always" (mpi_single.py: the new state is always kept) or
    "improve" (mpi_twins.py: kept only if the score improves); default by mode.
    check_disjoint: debug mode, assert that each round's blocks are a
    partition (no child in two blocks; twins: no pair overlap), which the
    in-place apply relies on.
    pipeline: overlap round r's score with round r+1 (engines with
    score_begin; keep-if-improved rounds are speculated and re-run after a
    rejection); identical results and history, but `types`
    already holds round r+1 when on_round(r) runs, so an on_round that reads
    the state (a checkpoint) needs the serial loop.
    score_check_every: 0 = rescore the whole state every round (the
    reference); K > 0 = the delta all-reduce of SURVEY §8(e) with a full
    rescore every K rounds that must agree (see _Sums); default K = 16 at
    every N (same per-round sums either way).  sums0: the exact (S_child, S_gift) of the
    start state, if known (else one rescore)."""
    world = world or World()
    accept = accept or ("always" if mode == _lib.SH_MODE_SINGLE else "improve")
    if accept not in ("always", "improve"):
        raise ValueError(f"accept must be 'always' or 'improve', not {accept!r}")
    _, _, _, nb = engine.geometry(mode, n)
    B = nb if blocks_per_round is None else int(blocks_per_round)
    if B < 1 or B > nb:
        raise ValueError(f"blocks_per_round must be in [1, {nb}]")
    if mode != _lib.SH_MODE_SINGLE and blocks_per_round is not None and world.size > nb:
        # mpi_twins.py:128,132 indexes child_blocks[rank] -> IndexError there
        raise ValueError(f"{world.size} ranks > {nb} twin blocks per round (the reference "
                         "raises IndexError at mpi_twins.py:132)")
    res = LoopResult()
    sums = _Sums(engine, world, score_check_every, max_rounds)
    budget = getattr(engine, "set_round_budget", None)
    if budget is not None:
        budget(max_rounds)
    if getattr(engine, "error_flags", None) is not None:
        engine.error_flags()  # the flags cover this run only: drop what earlier calls left
    if sums0 is None and (score0 is None or sums.delta):
        sums0 = tuple(engine.score_sums(types)[:2])
    if score0 is None:
        score0 = engine.score_from_sums(*sums0)
    cur = sums0  # exact sums of the current (accepted) state, delta mode
    best = score0
    res.best_score = best
    count = 0
    buffers: dict = {}
    backup = torch.empty_like(types) if accept == "improve" else None
    b0, b1, _ = shard_range(B, world.rank, world.size)
    if pipeline and hasattr(engine, "score_begin"):
        res = _run_pipelined(engine, types, mode, n, B, seed, max_rounds, patience, world,
                             on_round, best, check_disjoint, res, accept, sums, cur)
        check_engine_errors(engine, world, types.device)
        sums.final_check(types, res.sums, res.history)
        _drain(engine)
        return res
    for rnd in range(max_rounds):
        t0 = time.perf_counter()
        rows, tok = _sample(engine, mode, n, B, seed, rnd, types)
        if check_disjoint:
            assert_disjoint(rows, mode)
        if backup is not None and tok is None:
            backup.copy_(types)
        d = sums.buffer(0) if sums.delta else None
        _announce(engine, d, sums, world, rnd, snapshot=False)
        if b1 > b0:
            engine.solve_blocks(mode, rows[b0 * n:b1 * n], n, types, delta=d)
        if world.distributed:
            exchange(engine, world, mode, rows, n, B, types, buffers,
                     _next_sampler(engine, mode, n, B, seed, rnd, max_rounds))
        if check_disjoint:
            check_engine_errors(engine, world, types.device)
        if sums.delta:
            sc, sg, bad_tri, bad_tw = sums.combine(
                cur, rnd, *engine.delta_begin(types, d, sums.check_round(rnd), after=sums.reduce(d),
                                              snapshot=False).result())
        else:
            sc, sg, bad_tri, bad_tw = engine.score_sums(types)
        if bad_tri or bad_tw:
            raise AssertionError("triplets/twins must share a gift (mpi_single.py:32-44)")
        score = engine.score_from_sums(sc, sg)
        improved = score > best
        if improved:
            best = score
            count = 0
        else:
            count += 1
        kept = True
        if accept == "improve" and not improved:
            if tok is not None:
                tok.undo(types)  # (the round's undo record: its blocks' starting types)
            else:
                types.copy_(backup)
            kept = False
        if kept:
            cur = (sc, sg)
        res.rounds += 1
        res.blocks_solved += B
        st = RoundStats(rnd, sc, sg, score, kept, best, B, time.perf_counter() - t0)
        res.history.append(st)
        if on_round is not None:
            on_round(st)
        if count > patience:
            break
    res.best_score = best
    res.sums = cur
    check_engine_errors(engine, world, types.device)
    sums.final_check(types, cur, res.history)
    _drain(engine)
    return res


def _sample(engine, mode, n, B, seed, rnd, types):
    """Round rnd's rows and, from engines with sample_round, its undo record
    (a token whose undo(types) restores the round's starting types at its
    rows: the round is undone without a copy of the whole state); (rows,
    None) from the others, which the loops roll back by copies."""
    sr = getattr(engine, "sample_round", None)
    if sr is None:
        return engine.sample_blocks(mode, n, B, seed, rnd), None
    return sr(mode, n, B, seed, rnd, types)


def _announce(engine, d, sums, world, rnd, snapshot) -> None:
    """Before a round's solve, tell an engine with a host mailbox
    (GPUEngine.announce_delta) how the round's delta d will be read -- the
    arguments its delta_begin will get -- so that the mailbox publish can
    ride on the round's last launch."""
    a = getattr(engine, "announce_delta", None)
    if a is not None and d is not None:
        a(d, sums.check_round(rnd), world.distributed, snapshot)


def _drain(engine) -> None:
    """Engines with side-stream work (GPUEngine.drain) finish it before the
    loop returns and its delta buffers are released."""
    d = getattr(engine, "drain", None)
    if d is not None:
        d()


def _run_pipelined(engine, types, mode, n, B, seed, max_rounds, patience, world, on_round, best,
                   check_disjoint, res: LoopResult, accept: str, sums: _Sums, cur) -> LoopResult:
    """run_rounds with round r's score overlapped with round r+1 (see the
    module docstring); same decisions, history and final state as the serial
    loop.  Round r+1 is launched speculatively from round r's result.  When
    round r turns out rejected (accept="improve": twins, triplets) the state
    goes back to round r's starting snapshot and round r+1 is run again from
    it; when the stop rule fires, the speculative round is undone."""
    b0, b1, _ = shard_range(B, world.rank, world.size)
    buffers: dict = {}
    improve = accept == "improve"
    undo_mode = getattr(engine, "sample_round", None) is not None
    # rollback targets: each round's undo record (undo_mode), or a copy of its
    # starting state
    pre = [torch.empty_like(types) for _ in range(2)] if improve and not undo_mode else None
    tok = [None, None]
    count = 0
    pending = None  # (round, score handle, start time, pre slot) of the round awaiting its score
    stop = False
    rnd = 0

    def launch(r: int, k: int):
        if pre is not None:
            pre[k].copy_(types)  # round r's starting state (its rollback target)
        rows, tok[k] = _sample(engine, mode, n, B, seed, r, types)
        if check_disjoint:
            assert_disjoint(rows, mode)
        d = sums.buffer(k) if sums.delta else None
        _announce(engine, d, sums, world, r, snapshot=not undo_mode)
        if b1 > b0:
            engine.solve_blocks(mode, rows[b0 * n:b1 * n], n, types, delta=d)
        if world.distributed:
            exchange(engine, world, mode, rows, n, B, types, buffers,
                     _next_sampler(engine, mode, n, B, seed, r, max_rounds))
        if check_disjoint:
            check_engine_errors(engine, world, types.device)
        if sums.delta:  # (a snapshot only for a check round's rescore, or for the copy rollback)
            return engine.delta_begin(types, d, sums.check_round(r), after=sums.reduce(d),
                                      snapshot=not undo_mode)
        return engine.score_begin(types)

    while True:
        if pending is None and (stop or rnd >= max_rounds):
            break
        t0 = time.perf_counter()
        handle = None
        k = rnd & 1
        if not stop and rnd < max_rounds:
            handle = launch(rnd, k)
        if pending is not None:
            prnd, ph, pt0, pk = pending
            if sums.delta:  # (a rejected round's successor re-runs from the same start state)
                sc, sg, bad_tri, bad_tw = sums.combine(cur, prnd, *ph.result())
            else:
                sc, sg, bad_tri, bad_tw = ph.result()
            if bad_tri or bad_tw:
                raise AssertionError("triplets/twins must share a gift (mpi_single.py:32-44)")
            score = engine.score_from_sums(sc, sg)
            improved = score > best
            if improved:
                best = score
                count = 0
            else:
                count += 1
            kept = improved or not improve
            if not kept:  # the state after round prnd is its starting state
                if undo_mode:
                    if handle is not None:
                        tok[k].undo(types)  # the speculative round rnd first
                    tok[pk].undo(types)
                else:
                    types.copy_(pre[pk])
            else:
                cur = (sc, sg)
            res.rounds += 1
            res.blocks_solved += B
            st = RoundStats(prnd, sc, sg, score, kept, best, B, t0 - pt0)
            res.history.append(st)
            if on_round is not None:
                on_round(st)
            if count > patience:
                stop = True
            if handle is not None:
                if stop:  # the serial loop ends after round prnd: undo the speculative round
                    if kept:
                        if undo_mode:
                            tok[k].undo(types)
                        else:
                            ph.restore(types)
                    handle = None
                elif not kept:  # round rnd ran from a rejected state: run it again
                    handle = launch(rnd, k)
        pending = (rnd, handle, t0, k) if handle is not None else None
        rnd += 1
    res.best_score = best
    res.sums = cur
    return res


def _next_sampler(engine, mode, n, B, seed, rnd, max_rounds):
    """The exchange's `during` work: round rnd + 1's blocks, sampled while
    round rnd's all-gather runs (engines with prefetch_blocks).  None after
    the last round of the budget (no round rnd + 1 will run; a patience stop
    cannot be known in advance, so that one round's sampling is spent)."""
    pf = getattr(engine, "prefetch_blocks", None)
    if pf is None or rnd + 1 >= max_rounds:
        return None
    return lambda: pf(mode, n, B, seed, rnd + 1)


def assert_disjoint(rows: torch.Tensor, mode: int) -> None:
    """Debug check: the round's blocks share no child.  Rows are
    first members c of units (c, .., c + mode): twins pairs, triplets."""
    r = rows.reshape(-1).long()
    kids = torch.cat([r + m for m in range(mode + 1)])
    if torch.unique(kids).numel() != kids.numel() or bool((r < 0).any()):
        raise AssertionError("blocks of a round are not disjoint (the in-place apply needs a partition)")


_ZEROED = object()  # GPUEngine._zero_ev: the delta was zeroed on the round's stream


def _wait_mail(mail, slot: int, seq: int, stream, busy: float = 0.1, poll: float = 20e-6,
               check_every: float = 5e-3):
    """Wait for mailbox slot `slot` to carry sequence number `seq`, then
    return its (dS_child, dS_gift, None).  A bounded wait, not a spin
    forever: every `check_every` seconds the publishing stream is queried,
    which raises a pending asynchronous HIP error (a faulted or aborted block
    kernel); once the stream is idle, every launch before the publish has run,
    so a sequence number still missing means the publish never happened (an
    announce/solve bookkeeping mismatch, a kernel that left early) and the
    wait raises instead of hanging.  Sequence numbers only grow per context:
    a larger one in the slot means this round's value was overwritten.
    The first `busy` seconds poll without sleeping: a round's publish lands
    within milliseconds, and a sleep's wake-up (tens of microseconds to
    milliseconds, by the host's timer slack) would be added to every round
    (round 6: a 256-iteration spin then 20 us sleeps cost the 6-block
    triplets round 1.5 -> 6.4 ms)."""
    t0 = time.perf_counter()
    next_check = t0 + check_every
    while True:
        got = mail[4 * slot]
        if got == seq:
            return int(mail[4 * slot + 1]), int(mail[4 * slot + 2]), None
        if got > seq:
            raise RuntimeError(f"mailbox slot {slot}: sequence {got} overwrote {seq} before it was read")
        now = time.perf_counter()
        if now >= next_check:
            # (query() raises a pending HIP error of the round's kernels; once
            #  it reports idle, the publish has landed if it ever will)
            if stream.query() and mail[4 * slot] != seq:
                raise RuntimeError(f"mailbox slot {slot}: the round's stream is idle but sequence {seq} "
                                   f"was never published (slot holds {mail[4 * slot]})")
            next_check = now + check_every
        if now - t0 > busy:
            time.sleep(poll)


def _wait(stream, ev) -> None:
    """stream waits for ev, unless ev has completed already (then a wait
    would only add a barrier packet between two block kernels)."""
    if not ev.query():
        stream.wait_event(ev)


class GPUEngine:
    """Adapter of SantaGPU to the run_rounds engine protocol.

    After the round's snapshot, the round's bookkeeping runs on a side
    stream, off the round's critical path: the delta sums' host copy (16
    bytes, after their all-reduce on N > 1 ranks), the rescore of check
    rounds, and the delta buffer's zeroing for its next round (a 16-byte
    fill).  The round's stream carries the sampling, the block kernels and
    the snapshot copy.  Sampling ahead on the side stream is available
    (PREFETCH, a ring of buffers: round r's blocks depend only on (seed,
    round r), A1) but measured slower (profiles/r04_gap_probe.json)."""

    def __init__(self, ctx):
        self.ctx = ctx
        self._pf_key = None
        self._zero_ev = {}
        self._cur = None     # (slot, round, mode, n, B, seed) of the round sample_round returned last
        self._budget = None  # rounds the loop runs (set_round_budget): no next-round sampling after the last

    def geometry(self, mode, n):
        return self.ctx.geometry(mode, n)

    def _side_stream(self):
        if not hasattr(self, "_side"):
            self._side = torch.cuda.Stream(self.ctx.device)
        return self._side

    # rounds sampled ahead on the side stream (ring of max(PREFETCH + 1, 2)
    # row buffers); 0 = on the round's stream, the default: a sampling kernel
    # beside the block kernel runs at its low issue priority for ~550 us and
    # cost the round 6-19 us more than the same kernel (~10 us) in line
    # (profiles/r04_gap_probe.json: loop_p0_* against loop_p2_*)
    PREFETCH = 0
    SIDE_STREAM = True  # the round's bookkeeping after the snapshot on the side stream
    # round r's block kernel samples round r + 1's rows (sh_solve_round) when
    # it solves the whole round (one GPU): a ring of three row buffers keeps
    # rounds r - 1 (a pending rollback), r and r + 1 apart
    FUSED_SAMPLING = True
    RING = 3

    def set_round_budget(self, max_rounds):
        """run_rounds' round budget: the last round samples no successor."""
        self._budget = max_rounds

    def sample_blocks(self, mode, n, B, seed, rnd):
        """Round rnd's block rows (A1): sampled on the round's stream (or
        already, by prefetch_blocks), or with PREFETCH = K > 0 taken from the
        side stream, where rounds rnd + 1 .. rnd + K are started (when the
        rounds come in order, round rnd was sampled while round rnd - K
        solved).  The returned buffer (one of max(K + 1, 2)) stays valid
        until round rnd + max(K + 1, 2) is asked for or prefetched (run_rounds
        uses it within its round)."""
        ring, main, k = self._ring(mode, n, B, seed, rnd)
        self._sample_into(mode, n, B, seed, rnd, main, k)
        free = None
        for j in range(rnd + 1, rnd + 1 + self.PREFETCH):
            s = j % ring
            if self._pf_rnd[s] == j:
                continue
            if free is None:
                free = torch.cuda.Event()
                free.record(main)  # (rounds <= rnd - 1, the last readers of buffer s, are enqueued)
            side = self._side_stream()
            with torch.cuda.stream(side):
                side.wait_event(free)
                self.ctx.sample_blocks(mode, n, B, seed, j, out=self._pf_buf[s])
                ev = torch.cuda.Event()
                ev.record(side)
            self._pf_rnd[s] = j
            self._pf_ev[s] = ev
        return self._pf_buf[k]

    def _ring(self, mode, n, B, seed, rnd):
        key = (mode, n, B, seed)
        ring = max(self.PREFETCH + 1, self.RING)
        if self._pf_key != key:
            self._pf_key = key
            self._pf_buf = [torch.empty(B * n, dtype=torch.int32, device=self.ctx.device) for _ in range(ring)]
            self._undo_buf = [torch.empty(B * n, dtype=torch.int16, device=self.ctx.device) for _ in range(ring)]
            self._pf_rnd = [None] * ring
            self._pf_ev = [None] * ring
            self._by_solve = [False] * ring  # rows sampled by the previous round's block kernel
        return ring, torch.cuda.current_stream(self.ctx.device), rnd % ring

    def _sample_into(self, mode, n, B, seed, rnd, main, k):
        if self._pf_ev[k] is not None:  # (a side-stream prefetch into buffer k: wait for it)
            _wait(main, self._pf_ev[k])
            self._pf_ev[k] = None
        if self._pf_rnd[k] != rnd:
            self.ctx.sample_blocks(mode, n, B, seed, rnd, out=self._pf_buf[k])
            self._pf_rnd[k] = rnd
            self._by_solve[k] = False

    def sample_round(self, mode, n, B, seed, rnd, types):
        """Round rnd's rows and its undo record (run_rounds' undo protocol):
        one launch samples the rows and gathers the round's starting types at
        them (sh_sample_blocks_undo), or, when the rows were sampled ahead
        (prefetch_blocks: N > 1, behind the previous round's all-gather and
        before its unpack), the types are gathered now (sh_pack_types).  The
        token's undo(types) scatters them back (sh_unpack_types).  The rows and
        undo record live in buffer rnd % RING of a ring of three: round rnd's
        block kernels sample round rnd + 1's rows into the next buffer
        (solve_blocks -> sh_solve_round), so the token stays valid until round
        rnd + 3 is sampled, i.e. until round rnd + 2's kernels run -- after
        every rollback the loops can ask for (the pipelined loop undoes round
        rnd while round rnd + 1 is in flight)."""
        ring, main, k = self._ring(mode, n, B, seed, rnd)
        rows, undo, cnt = self._pf_buf[k], self._undo_buf[k], B * n
        if self._pf_ev[k] is not None:
            _wait(main, self._pf_ev[k])
            self._pf_ev[k] = None
        # the undo record is gathered by this round's block kernels when they
        # solve the whole round (solve_blocks), else here
        self._cur = (k, rnd, mode, n, B, seed, self._pf_rnd[k] == rnd and self._by_solve[k])
        if self._pf_rnd[k] == rnd:
            if not self._cur[6]:
                self.ctx.pack_types(types, rows[:cnt], undo[:cnt])
        else:
            self.ctx.sample_blocks_undo(mode, n, B, seed, rnd, types, out=rows, undo=undo)
            self._pf_rnd[k] = rnd
            self._by_solve[k] = False
        ctx = self.ctx

        class _Undo:
            def undo(_, t):
                ctx.unpack_types(t, rows[:cnt], undo[:cnt], mode)
        return rows, _Undo()

    def prefetch_blocks(self, mode, n, B, seed, rnd):
        """Sample round rnd's blocks now, on the round's stream, for the next
        sample_blocks(rnd): the N > 1 loop calls it while the previous round's
        all-gather runs (exchange's `during`), so the sampling kernel overlaps
        the collective.  Buffer rnd % ring was last read by round rnd - ring
        (<= rnd - 2), enqueued on this stream before."""
        _, main, k = self._ring(mode, n, B, seed, rnd)
        self._sample_into(mode, n, B, seed, rnd, main, k)

    def zeroed_delta(self, d):
        """d, zeroed: by the side stream after its previous round's host copy
        (delta_begin), by its publish kernel on the round's stream (the
        mailbox), or here on the current stream the first time."""
        ev = self._zero_ev.pop(d.data_ptr(), None)
        if ev is None:
            d.zero_()
        elif ev is not _ZEROED:
            _wait(torch.cuda.current_stream(d.device), ev)
        return d

    def solve_blocks(self, mode, rows, n, types, delta=None, steps=None):
        """The round's blocks (or this rank's shard).  When the round came
        from sample_round and this call solves all of it (one GPU), the block
        kernels also write the round's undo record, if sample_round left it to
        them, and sample the next round's rows (sh_solve_round)."""
        cur = self._cur
        self._cur = None
        ann = self._announced
        self._announced = None
        full = (cur is not None and self.FUSED_SAMPLING and rows.numel() == cur[4] * n
                and rows.data_ptr() == self._pf_buf[cur[0]].data_ptr())
        if not full:
            if cur is not None and cur[6]:  # (the undo record was left to the kernels: gather it now)
                k = cur[0]
                self.ctx.pack_types(types, self._pf_buf[k][:cur[4] * n], self._undo_buf[k][:cur[4] * n])
            self.ctx.solve_blocks(mode, rows, n, types, delta=delta, steps=steps)
            return
        k, rnd, mode_, n_, B, seed, undo_pending = cur
        nxt = None
        if self._budget is None or rnd + 1 < self._budget:
            k1 = (rnd + 1) % len(self._pf_buf)
            if self._pf_rnd[k1] != rnd + 1 and self._pf_ev[k1] is None:
                nxt = (seed, rnd + 1, B, self._pf_buf[k1])
                self._pf_rnd[k1] = rnd + 1
                self._by_solve[k1] = True
        pub = None
        if ann is not None and delta is not None and ann == (delta.data_ptr(), True):
            pub = self._next_mail()
            self._prepub = (delta.data_ptr(),) + pub
        self.ctx.solve_round(mode, rows, n, types, undo=self._undo_buf[k] if undo_pending else None,
                             next_round=nxt, delta=delta, steps=steps, publish=pub)

    def new_delta(self):
        return torch.zeros(2, dtype=torch.int64, device=self.ctx.device)

    def pack_types(self, types, rows, out):
        self.ctx.pack_types(types, rows, out)

    def unpack_types(self, types, rows, vals, mode):
        self.ctx.unpack_types(types, rows, vals, mode)

    def score_sums(self, types):
        return self.ctx.score_sums(types)

    def error_flags(self):
        return self.ctx.error_flags()

    def drain(self):
        """End of a run: wait for the side stream's last work (the final
        round's delta copy and zeroing, a dropped speculative round's rescore)
        and forget the zeroing events, so that nothing of this run is pending
        on buffers the caller frees or on the next run's first round."""
        if hasattr(self, "_side"):
            self._side.synchronize()
        self._zero_ev.clear()

    def score_begin(self, types):
        """Snapshot `types` and score the snapshot on a side stream; returns a
        handle with result() -> score sums and restore(types) -> copy the
        snapshot back (pipelined rounds)."""
        return self._begin(types, None, True)

    def delta_begin(self, types, d, full: bool, after=None, snapshot: bool = True):
        """Delta rounds: copy the delta d to the host (once `after`, its
        all-reduce's work handle, is done) and, if `full`, rescore a snapshot
        of `types` on the side stream; result() -> (dS_child, dS_gift, full
        sums or None).  snapshot=False (the undo protocol, sample_round): no
        snapshot unless `full` -- no 2 MB copy on the round's stream -- and
        the handle cannot restore()."""
        return self._begin(types, d, full, after, snapshot)

    # one GPU, a round with neither rescore nor snapshot: its delta sums reach
    # the host through the context's mailbox (one one-lane kernel after the
    # round's kernels, polled by the host) instead of an event, a second
    # stream's copy and a cross-stream wait between two rounds' kernels
    MAILBOX = True
    _announced = None  # (delta address, read through the mailbox) of the next solve
    _prepub = None  # (delta address, slot, seq) published by the last solve_round

    def announce_delta(self, d, full: bool, reduced: bool, snapshot: bool):
        """The loop's delta_begin arguments for the round about to be solved
        (run_rounds' _announce): a mailbox round solved whole by one
        solve_round call publishes from that call's last launch (the fallback
        launch's last workgroup), one launch fewer between two rounds."""
        self._announced = (d.data_ptr(), bool(self.MAILBOX and not (full or reduced or snapshot)))

    def _next_mail(self):
        ctx = self.ctx
        slot = getattr(self, "_mslot", 0)
        self._mslot = slot ^ 1
        seq = getattr(ctx, "_mail_seq", 0) + 1  # (per context: unique across engines)
        ctx._mail_seq = seq
        return slot, seq

    def _publish(self, d):
        pre = self._prepub
        self._prepub = None
        if pre is not None and pre[0] == d.data_ptr():
            slot, seq = pre[1:]
        else:
            slot, seq = self._next_mail()
            self.ctx.publish_delta(d, slot, seq)
        self._zero_ev[d.data_ptr()] = _ZEROED  # (zeroed by the publish, in stream order)
        mail = self.ctx.mailbox
        stream = torch.cuda.current_stream(d.device)

        class _Handle:
            def result(_):
                return _wait_mail(mail, slot, seq, stream)

            def restore(_, t):
                raise RuntimeError("no snapshot was taken for this round (undo protocol)")
        return _Handle()

    def _begin(self, types, d, full: bool, after=None, snapshot: bool = True):
        if self.MAILBOX and d is not None and after is None and not (full or snapshot):
            return self._publish(d)
        if self._prepub is not None and d is not None and self._prepub[0] == d.data_ptr():
            raise RuntimeError("delta_begin: the round's delta was already published to the mailbox "
                               "(announce_delta announced a mailbox round)")
        if not hasattr(self, "_snaps"):
            dev = types.device
            self._side_stream()
            self._snaps = [torch.empty_like(types) for _ in range(2)]
            self._sums = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(2)]
            self._host = [torch.zeros(4, dtype=torch.int64).pin_memory() for _ in range(2)]
            self._dhost = [torch.zeros(2, dtype=torch.int64).pin_memory() for _ in range(2)]
            self._done = [None, None]
            self._k = 0
        k = self._k
        self._k ^= 1
        main = torch.cuda.current_stream(types.device)
        snap = self._snaps[k]
        if snapshot or full:
            if self._done[k] is not None:
                _wait(main, self._done[k])  # the score two rounds back has read the snapshot
            snap.copy_(types)
        dhost = self._dhost[k]
        side = self._side if self.SIDE_STREAM else main
        # everything after the snapshot runs on the side stream: the delta's
        # host copy and zeroing, the rescore (round 4: the host copy had been
        # on the round's stream, one more launch between two block kernels)
        with torch.cuda.stream(side):
            if side is not main:
                ready = torch.cuda.Event()
                ready.record(main)
                side.wait_event(ready)
            if after is not None:
                after.wait()  # (the side stream waits for the all-reduce of d)
            if d is not None:
                if side is not main:  # (the allocator must not recycle d under the side stream's work)
                    d.record_stream(side)
                dhost.copy_(d, non_blocking=True)
            if full:
                self.ctx.score_sums_async(snap, out=self._sums[k])
                self._host[k].copy_(self._sums[k], non_blocking=True)
            done = torch.cuda.Event()
            done.record(side)
            if d is not None:  # zeroed for its next round (zeroed_delta)
                d.zero_()
                if side is not main:
                    z = torch.cuda.Event()
                    z.record(side)
                    self._zero_ev[d.data_ptr()] = z
        self._done[k] = done
        host = self._host[k]

        class _Handle:
            def result(_):
                done.synchronize()
                sums = tuple(int(x) for x in host.tolist()) if full else None
                if d is None:
                    return sums
                return int(dhost[0]), int(dhost[1]), sums

            def restore(_, t):
                if not (snapshot or full):
                    raise RuntimeError("no snapshot was taken for this round (undo protocol)")
                torch.cuda.current_stream(t.device).wait_event(done)
                t.copy_(snap)
        return _Handle()

    def score_from_sums(self, sc, sg):
        from .context import score_from_sums
        c = self.ctx
        return score_from_sums(sc, sg, c.nc, c.ng, c.n_wish, c.n_good)


MODES = {"single": _lib.SH_MODE_SINGLE, "twins": _lib.SH_MODE_TWINS, "triplets": _lib.SH_MODE_TRIPLETS}


def my_optimizer(subm, score_org, comm=None, rank: int = 0, size: int = 1, gift_data=None,
                 child_data=None, *, mode: str = "single", block_size: int = 256,
                 blocks_per_round: int | None = None, seed: int = 2017, max_rounds: int = 100,
                 patience: int = 3, device: int = 0, verbose: bool = True):
    """Same call shape as the reference's my_optimizer (mpi_single.py:110).

    subm: DataFrame with ChildId, GiftId; gift_data = good-kids, child_data =
    wishlists (the reference's names).  `comm` is a torch.distributed
    process group (or None for one rank).  block_size counts rows: children
    for singles, twin pairs for twins, triplet units for mode="triplets"
    (an extension).  Returns the improved DataFrame."""
    from .context import SantaGPU
    ctx = SantaGPU(child_data, gift_data, child_data.shape[0] // gift_data.shape[0], device)
    # int64 first: a GiftId outside [0, ng) (or a child left at -1) must raise,
    # as the reference's indexing does, not wrap into int16
    types_np = np.full(ctx.nc, -1, dtype=np.int64)
    types_np[subm["ChildId"].to_numpy()] = subm["GiftId"].to_numpy()
    types = ctx.upload_types(types_np)
    m = MODES[mode]

    def log(st: RoundStats):
        if verbose and rank == 0:
            print("iteration:{} score achieved is: {:.10f}".format(st.round, st.best), flush=True)

    run_rounds(GPUEngine(ctx), types, mode=m, n=block_size, blocks_per_round=blocks_per_round,
               seed=seed, max_rounds=max_rounds, patience=patience,
               world=World(rank, size, comm), on_round=log, score0=score_org, pipeline=True)
    out = subm.copy()
    out["GiftId"] = types.cpu().numpy().astype(np.int64)[out["ChildId"].to_numpy()]
    return out


def main(argv=None) -> int:
    """CLI of the reference scripts (which take no arguments: every knob was
    a module global, mpi_single.py:193-240)."""
    ap = argparse.ArgumentParser(description="MI355X block-Hungarian optimiser (Santa 2017)")
    ap.add_argument("--mode", choices=list(MODES), default="single",
                    help="singles (mpi_single.py), twin pairs (mpi_twins.py) or triplet units (extension)")
    ap.add_argument("--block-size", type=int, default=256,
                    help="rows per block (pairs for twins, units for triplets)")
    ap.add_argument("--blocks-per-round", default="full",
                    help="'full' (all disjoint blocks), 'ranks' (reference: one per rank) or an int")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--patience", type=int, default=3)
    ap.add_argument("--accept", choices=["always", "improve"], default=None,
                    help="keep every round (mpi_single.py) or only improving ones (mpi_twins.py); "
                         "default by mode")
    ap.add_argument("--checkpoint-every", type=int, default=0, metavar="K",
                    help="rank 0 rewrites --out every K rounds (the reference: every round, "
                         "mpi_single.py:177)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="score each round before starting the next (default: overlapped, "
                         "same results)")
    ap.add_argument("--check-disjoint", action="store_true",
                    help="debug: assert every round's blocks are a partition")
    ap.add_argument("--seed", type=int, default=2017)
    ap.add_argument("--wishlist", help="child_wishlist_v2.csv (default: synthetic data)")
    ap.add_argument("--goodkids", help="gift_goodkids_v2.csv")
    ap.add_argument("--init", help="baseline_res.csv / improved_sub.csv to start from")
    ap.add_argument("--out", default=None, help="write the final submission CSV (rank 0)")
    ap.add_argument("--synthetic-seed", type=int, default=2017)
    args = ap.parse_args(argv)

    import os
    from .context import SantaGPU
    from . import data as D
    world = World()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        world = World(dist.get_rank(), dist.get_world_size(), None)
    dev = torch.cuda.current_device()
    if args.wishlist:
        wish, good = D.read_wishlist(args.wishlist), D.read_goodkids(args.goodkids)
        types0 = D.read_submission(args.init, wish.shape[0], good.shape[0])
        nq = wish.shape[0] // good.shape[0]
    else:
        sd = D.synthetic(args.synthetic_seed)
        wish, good, types0, nq = sd.wish, sd.goodkids, sd.types, sd.nq
        if args.init:
            types0 = D.read_submission(args.init, wish.shape[0], good.shape[0])
    ctx = SantaGPU(wish, good, nq, dev)
    types = ctx.upload_types(types0)
    mode = MODES[args.mode]
    bpr = None if args.blocks_per_round == "full" else (
        world.size if args.blocks_per_round == "ranks" else int(args.blocks_per_round))

    if args.checkpoint_every and not args.out:
        ap.error("--checkpoint-every needs --out")

    def log(st: RoundStats):
        if world.rank == 0:
            print(json.dumps(st.__dict__), flush=True)
            # the reference's per-round checkpoint (mpi_single.py:176-177), taken
            # after the round's timing: the accepted state is the current one
            if args.checkpoint_every and (st.round + 1) % args.checkpoint_every == 0:
                D.write_submission(args.out, types.cpu().numpy())

    res = run_rounds(GPUEngine(ctx), types, mode=mode, n=args.block_size, blocks_per_round=bpr,
                     seed=args.seed, max_rounds=args.rounds, accept=args.accept,
                     patience=args.patience, world=world, on_round=log,
                     check_disjoint=args.check_disjoint,
                     # (a checkpoint is taken in on_round: it needs the serial loop's state)
                     pipeline=not (args.no_pipeline or args.checkpoint_every))
    if world.rank == 0:
        print(json.dumps({"rounds": res.rounds, "blocks": res.blocks_solved,
                          "best_score": res.best_score}), flush=True)
        if args.out:
            D.write_submission(args.out, types.cpu().numpy())
    return 0


if __name__ == "__main__":
    sys.exit(main())

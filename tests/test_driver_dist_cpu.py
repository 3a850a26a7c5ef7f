"""Multi-rank driver logic on the CPU (gloo, world_size 2 and 3).

The product exchange (santa_hip.driver.exchange: shard -> pack -> one
all-gather -> unpack) and round loop run with the oracle-backed CPU engine;
the final assignment and every per-round score must equal the single-rank
run bit for bit (blocks are disjoint, integer sums are order-free), including
block counts that do not divide evenly across ranks, the twins rollback and
the triplet extension (mode 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from santa_hip import _lib
from santa_hip import data as D
from santa_hip.driver import World, run_rounds, shard_range

SMALL = dict(seed=3, nc=60000, ng=60, nq=1000, n_wish=20, n_good=300)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(eng_data, mode, n, bpr, rounds, world=None):
    from cpu_engine import CPUOracleEngine
    sd = eng_data
    eng = CPUOracleEngine(sd.wish, sd.goodkids, sd.nq)
    types = torch.from_numpy(sd.types.copy())
    res = run_rounds(eng, types, mode=mode, n=n, blocks_per_round=bpr, seed=17,
                     max_rounds=rounds, world=world or World(), patience=100)
    assert eng.drained == 1  # (the loop drains the engine's side work once, at its end)
    return types.numpy().copy(), [st.score for st in res.history], list(eng.prefetched)


def _worker(rank, size, port, mode, n, bpr, rounds, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "mpi-hungarian-method_amd"), os.path.join(root, "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    sd = D.synthetic(**SMALL)
    out[rank] = _run(sd, mode, n, bpr, rounds, World(rank, size, None))
    dist.destroy_process_group()


@pytest.mark.parametrize("size,mode,n,bpr", [(2, 0, 64, None), (3, 0, 100, 7), (2, 1, 16, None),
                                              (2, 2, 16, None)])
def test_multirank_equals_single_rank(size, mode, n, bpr):
    sd = D.synthetic(**SMALL)
    rounds = 3
    ref_t, ref_scores, _ = _run(sd, mode, n, bpr, rounds)
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(size, port, mode, n, bpr, rounds, out), nprocs=size, join=True)
    for r in range(size):
        t, scores, pref = out[r]
        assert np.array_equal(t, ref_t), f"rank {r} state differs"
        assert scores == ref_scores
        # the exchange samples the next round behind the all-gather, but not
        # after the budget's last round (no round `rounds` runs)
        assert pref == list(range(1, rounds)), pref


def test_shard_range_covers_blocks():
    for B in (1, 7, 78, 3730):
        for size in (1, 2, 3, 4, 8):
            seen = []
            for r in range(size):
                b0, b1, per = shard_range(B, r, size)
                assert b1 - b0 <= per
                seen.extend(range(b0, b1))
            assert seen == list(range(B))


def test_twins_rank_limit_matches_reference():
    """mpi_twins.py:128,132 raises IndexError with more ranks than twin
    blocks; the reference-schedule driver refuses that configuration."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)
    eng = CPUOracleEngine(sd.wish, sd.goodkids, sd.nq)
    _, _, _, nb = eng.geometry(_lib.SH_MODE_TWINS, 64)
    with pytest.raises(ValueError):
        run_rounds(eng, torch.from_numpy(sd.types.copy()), mode=_lib.SH_MODE_TWINS, n=64,
                   blocks_per_round=1, world=World(0, nb + 1, None), max_rounds=1)


def test_all_gather_sends_rccl_dtypes(monkeypatch):
    """torch's NCCL/RCCL process group has no int16 datatype: the int16 type
    vectors must reach the collective as bytes (uint8), not as int16."""
    from santa_hip.driver import all_gather_flat
    seen = []

    def fake(out, inp, group=None, async_op=False):
        seen.append((out.dtype, inp.dtype))
        out.copy_(inp.repeat(out.numel() // inp.numel()))

    monkeypatch.setattr(dist, "all_gather_into_tensor", fake)
    inp = torch.arange(-5, 5, dtype=torch.int16)
    out = torch.empty(20, dtype=torch.int16)
    all_gather_flat(out, inp)
    assert seen == [(torch.uint8, torch.uint8)]
    assert torch.equal(out, torch.cat([inp, inp]))


def test_accept_modes_and_disjoint_check():
    """--accept overrides the mode's rule (always-keep vs keep-if-improved),
    an unknown rule is refused, and the debug partition check passes on the
    sampler's blocks but catches an overlap."""
    from cpu_engine import CPUOracleEngine
    from santa_hip.driver import assert_disjoint
    sd = D.synthetic(**SMALL)
    eng = CPUOracleEngine(sd.wish, sd.goodkids, sd.nq)
    for accept in ("always", "improve"):
        t = torch.from_numpy(sd.types.copy())
        res = run_rounds(eng, t, mode=_lib.SH_MODE_SINGLE, n=64, seed=3, max_rounds=2,
                         accept=accept, world=World(), check_disjoint=True)
        assert res.rounds == 2
        assert all(st.accepted for st in res.history) or accept == "improve"
    with pytest.raises(ValueError):
        run_rounds(eng, torch.from_numpy(sd.types.copy()), mode=0, n=64, max_rounds=1, accept="maybe")
    rows = eng.sample_blocks(_lib.SH_MODE_TWINS, 16, 4, 1, 0)
    assert_disjoint(rows, _lib.SH_MODE_TWINS)
    with pytest.raises(AssertionError):
        assert_disjoint(torch.cat([rows, rows[:1]]), _lib.SH_MODE_TWINS)
    with pytest.raises(AssertionError):  # pairs (c, c+1) and (c+1, c+2) overlap
        assert_disjoint(torch.tensor([11, 12], dtype=torch.int32), _lib.SH_MODE_TWINS)


@pytest.mark.parametrize("mode,n,accept,warm", [(0, 64, None, 0), (1, 16, None, 0), (2, 16, None, 0),
                                                (0, 64, "improve", 0), (1, 16, None, 12), (2, 8, None, 12)])
@pytest.mark.parametrize("patience,rounds", [(-1, 4), (0, 6), (1, 8), (100, 3), (100, 0)])
def test_pipelined_rounds_equal_serial(mode, n, accept, warm, patience, rounds):
    """The pipelined loop (round r's score overlapped with round r+1: a
    speculative round undone when the stop rule fires, re-run when round r
    is rejected under keep-if-improved) makes the same decisions, history and
    final state as the serial loop."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)
    start = torch.from_numpy(sd.types.copy())
    if warm:  # a converged state, where keep-if-improved rounds get rejected
        run_rounds(CPUOracleEngine(sd.wish, sd.goodkids, sd.nq), start, mode=mode, n=n, seed=99,
                   max_rounds=warm, patience=100, world=World())
    r0, _ = _serial_vs_pipelined(sd, start, mode, n, accept, patience, rounds)
    if patience == -1:
        assert r0 == 1  # stopped after the first round; the speculative second was undone


def _serial_vs_pipelined(sd, start, mode, n, accept, patience, rounds):
    """Run both loops from `start`, each with the undo protocol (rollbacks and
    the speculative round undone from each round's undo record) and with
    whole-state copies (an engine without sample_round); assert identical
    state, history and counts; return (rounds run, whether any round was
    rejected)."""
    from cpu_engine import CPUOracleEngine

    class Copies(CPUOracleEngine):
        sample_round = None  # (the loops fall back to snapshots and copies)

    out = []
    for pipeline in (False, True):
        for cls in (CPUOracleEngine, Copies):
            eng = cls(sd.wish, sd.goodkids, sd.nq)
            t = start.clone()
            res = run_rounds(eng, t, mode=mode, n=n, seed=5, max_rounds=rounds, accept=accept,
                             patience=patience, world=World(), pipeline=pipeline)
            assert (eng.undo_tokens > 0) == (cls is CPUOracleEngine and rounds > 0)
            hist = [(st.round, st.s_child, st.s_gift, st.score, st.accepted, st.best) for st in res.history]
            out.append((t.numpy().copy(), hist, res.rounds, res.blocks_solved, res.best_score))
    t0, h0, r0, b0, s0 = out[0]
    for t1, h1, r1, b1, s1 in out[1:]:
        assert np.array_equal(t0, t1)
        assert h0 == h1 and r0 == r1 and b0 == b1 and s0 == s1
    return r0, any(not a for (_, _, _, _, a, _) in h0)


@pytest.mark.parametrize("warm", [12, 40])
def test_pipelined_rejections_are_exercised(warm):
    """The re-run-after-rejection path of the pipelined loop, on its own: from
    a converged triplet state (warm rounds; on this small instance twins keep
    improving, triplets do not) keep-if-improved rounds get rejected, and the
    pipelined loop still equals the serial one."""
    mode, n = _lib.SH_MODE_TRIPLETS, 8
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)
    start = torch.from_numpy(sd.types.copy())
    run_rounds(CPUOracleEngine(sd.wish, sd.goodkids, sd.nq), start, mode=mode, n=n, seed=99,
               max_rounds=warm, patience=100, world=World())
    _, rejected = _serial_vs_pipelined(sd, start, mode, n, None, 100, 8)
    assert rejected, "no round was rejected: the re-run path was not exercised"


def test_triplet_rounds_keep_units():
    """Triplet rounds (mode 2, keep-if-improved): units move whole, so every
    triplet still shares a gift, and a rejected round leaves the state as it was."""
    from cpu_engine import CPUOracleEngine
    from santa_hip.driver import assert_disjoint
    sd = D.synthetic(**SMALL)
    eng = CPUOracleEngine(sd.wish, sd.goodkids, sd.nq)
    _, _, stride, nb = eng.geometry(_lib.SH_MODE_TRIPLETS, 16)
    assert stride == 3 and nb == eng.n_triplets // 3 // 16
    t = torch.from_numpy(sd.types.copy())
    res = run_rounds(eng, t, mode=_lib.SH_MODE_TRIPLETS, n=16, seed=2, max_rounds=3,
                     world=World(), check_disjoint=True)
    fam = t.numpy()[:eng.n_triplets].reshape(-1, 3)
    assert (fam == fam[:, :1]).all()
    assert res.rounds >= 1 and res.best_score >= res.history[0].score or not res.history[0].accepted
    rows = eng.sample_blocks(_lib.SH_MODE_TRIPLETS, 16, 2, 1, 0)
    assert_disjoint(rows, _lib.SH_MODE_TRIPLETS)
    with pytest.raises(AssertionError):  # units (c, c+1, c+2) and (c+2, ...) overlap
        assert_disjoint(torch.tensor([3, 5], dtype=torch.int32), _lib.SH_MODE_TRIPLETS)


@pytest.mark.parametrize("pipeline,check", [(False, False), (True, False), (False, True), (True, True)])
def test_device_error_flags_raise(pipeline, check):
    """A block the device skipped (error flags set) is never accepted
    silently: run_rounds raises at its end, and after the round itself with
    --check-disjoint, in the serial and the pipelined loop."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)

    class Flagged(CPUOracleEngine):
        rounds_solved = 0

        def solve_blocks(self, *a, **kw):
            self.rounds_solved += 1
            return super().solve_blocks(*a, **kw)

        def error_flags(self):
            return _lib.SH_ERRF_TYPE

    eng = Flagged(sd.wish, sd.goodkids, sd.nq)
    with pytest.raises(RuntimeError, match="error flags"):
        run_rounds(eng, torch.from_numpy(sd.types.copy()), mode=0, n=64, seed=1, max_rounds=3,
                   patience=100, world=World(), pipeline=pipeline, check_disjoint=check)
    assert eng.rounds_solved == (1 if check else 3)


@pytest.mark.parametrize("mode,n", [(0, 64), (1, 16), (2, 8)])
@pytest.mark.parametrize("pipeline", [False, True])
@pytest.mark.parametrize("every", [1, 3])
def test_delta_sums_equal_full_rescore(mode, n, pipeline, every):
    """SURVEY §8(e)'s delta all-reduce (each round's sums = the start state's
    + the blocks' exact deltas; a full rescore every K rounds must agree)
    gives the full-rescore loop's history, decisions and state, including
    keep-if-improved rollbacks (from a converged state) and the pipelined loop."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)
    start = torch.from_numpy(sd.types.copy())
    run_rounds(CPUOracleEngine(sd.wish, sd.goodkids, sd.nq), start, mode=mode, n=n, seed=99,
               max_rounds=12, patience=100, world=World())
    out = []
    for k in (0, every):
        t = start.clone()
        res = run_rounds(CPUOracleEngine(sd.wish, sd.goodkids, sd.nq), t, mode=mode, n=n, seed=5,
                         max_rounds=7, patience=2, world=World(), pipeline=pipeline, score_check_every=k)
        out.append((t.numpy().copy(), [(st.round, st.s_child, st.s_gift, st.score, st.accepted, st.best)
                                       for st in res.history]))
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


@pytest.mark.parametrize("pipeline", [False, True])
def test_delta_mismatch_raises(pipeline):
    """A delta that disagrees with the full rescore stops the run at the
    first check round."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)

    class Off(CPUOracleEngine):
        def solve_blocks(self, mode, rows, n, types, delta=None):
            super().solve_blocks(mode, rows, n, types, delta=delta)
            if delta is not None:
                delta[1] += 1

    with pytest.raises(RuntimeError, match="full rescore"):
        run_rounds(Off(sd.wish, sd.goodkids, sd.nq), torch.from_numpy(sd.types.copy()), mode=0, n=64,
                   seed=1, max_rounds=5, patience=100, world=World(), pipeline=pipeline,
                   score_check_every=2)


@pytest.mark.parametrize("pipeline", [False, True])
def test_patience_stop_is_checked_against_a_full_rescore(pipeline):
    """A run that stops on patience before its next check round still ends
    with a full rescore of the final state: a wrong delta cannot reach the
    final sums unverified (K larger than the rounds the run lasts)."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)

    class Off(CPUOracleEngine):
        def solve_blocks(self, mode, rows, n, types, delta=None):
            super().solve_blocks(mode, rows, n, types, delta=delta)
            if delta is not None:
                delta[1] += 1

    with pytest.raises(RuntimeError, match="final state"):
        run_rounds(Off(sd.wish, sd.goodkids, sd.nq), torch.from_numpy(sd.types.copy()), mode=0, n=64,
                   seed=1, max_rounds=50, patience=-1, world=World(), pipeline=pipeline,
                   score_check_every=40)
    # an honest engine passes the same final check and reports the final sums
    eng = CPUOracleEngine(sd.wish, sd.goodkids, sd.nq)
    t = torch.from_numpy(sd.types.copy())
    res = run_rounds(eng, t, mode=1, n=16, seed=1, max_rounds=50, patience=-1, world=World(),
                     pipeline=pipeline, score_check_every=40)
    assert res.rounds == 1
    assert res.sums == tuple(eng.score_sums(t)[:2])


def test_stale_error_flags_do_not_fail_a_new_run():
    """Flags left by an earlier, unrelated call on the same engine are read and
    dropped when run_rounds starts; flags raised during the run still fail it."""
    from cpu_engine import CPUOracleEngine
    sd = D.synthetic(**SMALL)

    class Stale(CPUOracleEngine):
        pending = _lib.SH_ERRF_TYPE

        def error_flags(self):
            f, self.pending = self.pending, 0
            return f

    eng = Stale(sd.wish, sd.goodkids, sd.nq)
    res = run_rounds(eng, torch.from_numpy(sd.types.copy()), mode=0, n=64, seed=1, max_rounds=2,
                     patience=100, world=World())
    assert res.rounds == 2


def _flag_worker(rank, size, port, pipeline, check, out):
    import datetime
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "mpi-hungarian-method_amd"), os.path.join(root, "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    from cpu_engine import CPUOracleEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size, timeout=datetime.timedelta(seconds=60))
    sd = D.synthetic(**SMALL)

    class OneRankFlags(CPUOracleEngine):
        solved = 0

        def solve_blocks(self, *a, **kw):
            self.solved += 1
            return super().solve_blocks(*a, **kw)

        def error_flags(self):  # only rank 1's device saw a bad block, from its first round on
            return _lib.SH_ERRF_TYPE if rank == 1 and self.solved else 0

    eng = OneRankFlags(sd.wish, sd.goodkids, sd.nq)
    try:
        run_rounds(eng, torch.from_numpy(sd.types.copy()), mode=0, n=64, seed=1, max_rounds=3,
                   patience=100, world=World(rank, size, None), pipeline=pipeline, check_disjoint=check)
        out[rank] = ("ok", eng.solved)
    except RuntimeError as e:
        out[rank] = (str(e), eng.solved)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipeline,check", [(False, True), (True, True), (False, False), (True, False)])
def test_error_flags_agreed_across_ranks(pipeline, check):
    """Only one rank's device flags a skipped block: every rank raises at the
    same point (the flags are all-reduced before anyone raises), so no rank is
    left waiting in a collective (the 60 s gloo timeout would fail this)."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_flag_worker, args=(2, port, pipeline, check, out), nprocs=2, join=True)
    for r in range(2):
        msg, solved = out[r]
        assert "error flags 0x4" in msg, (r, msg)
        assert solved == (1 if check else 3), (r, solved)


def test_mailbox_wait_is_bounded():
    """GPUEngine's mailbox wait (driver._wait_mail): returns the published
    sums, raises when the stream went idle without the publish, raises when a
    later sequence number overwrote the slot, and surfaces a stream error --
    instead of spinning forever."""
    from santa_hip.driver import _wait_mail

    class Stream:
        def __init__(self, idle=True, exc=None):
            self.idle, self.exc, self.calls = idle, exc, 0

        def query(self):
            self.calls += 1
            if self.exc:
                raise self.exc
            return self.idle

    mail = [0] * 8
    mail[4:8] = [7, 11, -3, 0]
    assert _wait_mail(mail, 1, 7, Stream()) == (11, -3, None)
    with pytest.raises(RuntimeError, match="never published"):
        _wait_mail(mail, 0, 5, Stream(idle=True), busy=0.0, poll=1e-5, check_every=1e-4)
    with pytest.raises(RuntimeError, match="overwrote"):
        _wait_mail(mail, 1, 6, Stream())
    with pytest.raises(ValueError, match="HIP error"):
        _wait_mail(mail, 0, 5, Stream(idle=False, exc=ValueError("HIP error")), busy=0.0, poll=1e-5,
                   check_every=1e-4)

    class Late(Stream):  # the publish lands while the stream is still busy
        def query(self):
            self.calls += 1
            if self.calls == 3:
                mail[0:3] = [9, 1, 2]
            return False
    assert _wait_mail(mail, 0, 9, Late(), busy=0.0, poll=1e-5, check_every=1e-4) == (1, 2, None)

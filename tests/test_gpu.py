"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors.  Integer/index results must be bit-exact."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402
from conftest import golden_json  # noqa: E402
from cpu_engine import sha  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sh():
    import santa_hip
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    return santa_hip


@pytest.fixture(scope="module")
def ctx(sh, full_data):
    return sh.SantaGPU.from_data(full_data, 0)


# --------------------------------------------------------------------------- LSAP
def test_lsap_golden_int(sh, lsap_cases):
    z, meta = lsap_cases
    by_n = {}
    for m in meta:
        if m["kind"] == "int":
            by_n.setdefault(m["n"], []).append(m)
    for n, ms in by_n.items():
        C = np.stack([z[f"C{m['i']}"].astype(np.int64) for m in ms])
        want = np.stack([z[f"col{m['i']}"].astype(np.int64) for m in ms])
        for dt in (torch.int64, torch.int32):
            col, cost = sh.solve_batched(torch.from_numpy(C).to("cuda", dt))
            assert np.array_equal(col.cpu().numpy(), want), (n, dt)
            assert cost.cpu().tolist() == [m["cost"] for m in ms]
        col, _ = sh.solve_batched(torch.from_numpy(C.astype(np.float64)).cuda())
        assert np.array_equal(col.cpu().numpy(), want), (n, "f64")


def test_lsap_golden_float(sh, lsap_cases):
    z, meta = lsap_cases
    for m in meta:
        if not m["kind"].startswith("f64"):
            continue
        C = torch.from_numpy(z[f"C{m['i']}"]).cuda()[None]
        col, cost = sh.solve_batched(C)
        want = z[f"col{m['i']}"].astype(np.int64)
        assert np.array_equal(col[0].cpu().numpy(), want), m
        if m["feasible"]:
            _, c2 = sh.linear_sum_assignment(z[f"C{m['i']}"])
            assert np.array_equal(c2, want)
        else:
            with pytest.raises(ValueError):
                sh.linear_sum_assignment(z[f"C{m['i']}"])


@pytest.mark.parametrize("n", [64, 128, 256, 512, 1024])
def test_lsap_random_vs_oracle(sh, n):
    rng = np.random.default_rng(n)
    B = 4 if n <= 256 else 2
    C = rng.integers(0, 1 << 16, size=(B, n, n), dtype=np.int64)
    col, cost = sh.solve_batched(torch.from_numpy(C).cuda())
    ocol, ocost = oracle.lsap_i64_batched(C)
    assert np.array_equal(col.cpu().numpy(), ocol)
    assert np.array_equal(cost.cpu().numpy(), ocost)


@pytest.mark.parametrize("n,mod", [(64, 3), (100, 1 << 16), (256, 1 << 16), (1000, 7)])
def test_lsap_hash_vs_oracle(sh, n, mod):
    from santa_hip.sampler import hash_matrix
    B = 3
    col, cost = sh.solve_hash(1234, mod, n, B)
    col = col.cpu().numpy()
    for b in range(B):
        C = hash_matrix(1234, b, n, mod)
        _, oc = oracle.lsap(C)
        assert np.array_equal(col[b], oc)
        assert int(cost[b]) == int(C[np.arange(n), oc].sum())


# --------------------------------------------------------------------------- sampler
@pytest.mark.parametrize("mode,n,B", [(0, 256, 3730), (1, 256, 78), (0, 100, 50), (2, 256, 6)])
def test_sampler_matches_host_mirror(sh, ctx, mode, n, B):
    from santa_hip.sampler import sample_blocks
    lo, count, stride, nb = ctx.geometry(mode, n)
    assert B <= nb
    rows = ctx.sample_blocks(mode, n, B, 77, 5).cpu().numpy()
    want = sample_blocks(77, 5, lo, count, stride, n, B).reshape(-1)
    assert np.array_equal(rows, want)
    assert np.unique(rows).size == rows.size


# --------------------------------------------------------------------------- blocks
def test_santa_blocks_golden(sh, ctx, full_data, santa_blocks):
    z, meta = santa_blocks
    for m in meta:
        k, n = m["i"], m["n"]
        rows = torch.from_numpy(z[f"rows{k}"]).cuda()
        types = ctx.upload_types(full_data.types)
        col = torch.empty(n, dtype=torch.int32, device="cuda")
        cost = torch.empty(1, dtype=torch.int64, device="cuda")
        mode = 0 if m["mode"] == "single" else 1
        ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost)
        assert np.array_equal(col.cpu().numpy(), z[f"col{k}"].astype(np.int32)), m
        assert int(cost.item()) == m["cost_units"], m
    assert ctx.error_flags() == 0


def test_triplet_blocks_golden(sh, ctx, full_data, santa_triplets):
    """Triplet units (extension): scipy's col_ind and the exact cost of the
    float32 ((h1 + h2) + h3) matrix (tests/golden/santa_triplets.npz)."""
    z, meta = santa_triplets
    for m in meta:
        k, n = m["i"], m["n"]
        types = ctx.upload_types(full_data.types)
        col = torch.empty(n, dtype=torch.int32, device="cuda")
        cost = torch.empty(1, dtype=torch.int64, device="cuda")
        ctx.solve_blocks(2, torch.from_numpy(z[f"rows{k}"]).cuda(), n, types, col=col, cost=cost)
        assert np.array_equal(col.cpu().numpy(), z[f"col{k}"].astype(np.int32)), m
        assert int(cost.item()) == m["cost_units"], m
        t = types.cpu().numpy()
        r = z[f"rows{k}"]
        assert (t[r] == t[r + 1]).all() and (t[r] == t[r + 2]).all()
    sh.init(full_data.wish, full_data.goodkids)
    import pandas as pd
    subm = pd.DataFrame({"ChildId": np.arange(full_data.nc), "GiftId": full_data.types.astype(np.int64)})
    m = meta[0]
    blk = z[f"rows{m['i']}"].astype(np.int64)
    cids, gids = sh.optimize_block_triplets(blk, subm)
    assert np.array_equal(cids, blk)
    assert np.array_equal(gids, full_data.types[blk][z[f"col{m['i']}"]].astype(np.int64))
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("patience", [-1, 100])
def test_pipelined_rounds_equal_serial_gpu(sh, ctx, full_data, patience):
    """GPUEngine.score_begin (score on a side stream from a snapshot, next
    round launched meanwhile, speculative round undone at the stop) gives the
    serial loop's history and final state on full 3730-block rounds."""
    from santa_hip.driver import GPUEngine, World, run_rounds
    out = []
    for pipeline in (False, True):
        types = ctx.upload_types(full_data.types)
        res = run_rounds(GPUEngine(ctx), types, mode=0, n=256, seed=8, max_rounds=3,
                         patience=patience, world=World(), pipeline=pipeline)
        torch.cuda.synchronize()
        out.append((types.cpu().numpy(), [(st.round, st.s_child, st.s_gift, st.score, st.best)
                                          for st in res.history], res.rounds))
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]
    assert out[0][2] == (1 if patience == -1 else 3)
    assert ctx.error_flags() == 0


def test_santa_blocks_golden_reference_sizes(sh, ctx, full_data):
    """The reference's optimize_block at its default 2000 and
    optimize_block_twins at 3000 pairs (golden, made from the reference)."""
    from conftest import load_npz_cases
    z, meta = load_npz_cases("santa_blocks_large.npz")
    for m in meta:
        k, n = m["i"], m["n"]
        types = ctx.upload_types(full_data.types)
        col = torch.empty(n, dtype=torch.int32, device="cuda")
        cost = torch.empty(1, dtype=torch.int64, device="cuda")
        ctx.solve_blocks(0 if m["mode"] == "single" else 1, torch.from_numpy(z[f"rows{k}"]).cuda(), n,
                         types, col=col, cost=cost)
        assert np.array_equal(col.cpu().numpy(), z[f"col{k}"].astype(np.int32)), m
        assert int(cost.item()) == m["cost_units"], m
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("mode,n,B", [(0, 256, 64), (0, 64, 40), (0, 100, 16), (1, 256, 8),
                                      (1, 37, 9),
                                      # large blocks (row rebuilt from the wishlist per step),
                                      # up to the reference's own sizes (mpi_single.py:238,
                                      # mpi_twins.py:244)
                                      (0, 257, 3), (0, 700, 2), (0, 1024, 2), (0, 2000, 2),
                                      (1, 300, 2), (1, 1500, 1), (1, 3000, 1),
                                      # the largest block the boundary accepts (SH_MAX_N_SANTA)
                                      (0, 4096, 1), (1, 4096, 1),
                                      # triplet units (extension; always the row-rebuild design)
                                      (2, 256, 6), (2, 100, 5), (2, 37, 4), (2, 555, 3)])
def test_round_vs_oracle(sh, ctx, full_data, mode, n, B):
    """Fused build+solve+apply on the GPU equals the CPU oracle: col, exact
    cost, the whole new type vector, and the happiness deltas."""
    from santa_hip import _lib
    rows = ctx.sample_blocks(mode, n, B, 2024, 1)
    t_host = full_data.types.copy()
    st = np.zeros(2, dtype=np.uint64)
    ocol, ocost = oracle.round_blocks(mode, full_data.wish, t_host, rows.cpu().numpy().reshape(B, n),
                                      stats=st, ng=full_data.ng)
    s0 = oracle.score_sums(full_data.wish, full_data.goodkids, full_data.types)
    s1 = oracle.score_sums(full_data.wish, full_data.goodkids, t_host)
    # singles n <= 256: the default for few blocks (LDS tile) and the forced
    # throughput kernel (sparse) are both checked
    # (SH_FLAG_TEST_RANGE: every block leaves its scaled-unit solver -- the
    # register-tile design for the fallback launch, the LDS-tile kernel for its
    # windowed-key re-solve -- the path of an out-of-range block)
    if mode == 0 and n <= 256:
        flag_sets = (0, _lib.SH_FLAG_SP_TILE, _lib.SH_FLAG_SP1,
                     _lib.SH_FLAG_SP_TILE | _lib.SH_FLAG_TEST_RANGE,
                     _lib.SH_FLAG_LDS_TILE, _lib.SH_FLAG_LDS_TILE | _lib.SH_FLAG_TEST_RANGE,
                     _lib.SH_FLAG_VT_TILE, _lib.SH_FLAG_VT_TILE | _lib.SH_FLAG_TEST_RANGE,
                     _lib.SH_FLAG_DT_TILE, _lib.SH_FLAG_DT_TILE | _lib.SH_FLAG_TEST_RANGE)
    elif mode == 1 and n <= 256:
        flag_sets = (0, _lib.SH_FLAG_TEST_RANGE)
    elif mode == 0 and n <= 2048:
        # the staged-row lattice kernel (default), the row-rebuild kernel
        # (forced), and every block through the lattice kernel's fallback launch
        flag_sets = (0, _lib.SH_FLAG_BIG_ROWS, _lib.SH_FLAG_TEST_RANGE)
    else:
        flag_sets = (0,)
    for fl in flag_sets:
        types = ctx.upload_types(full_data.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        delta = torch.zeros(2, dtype=torch.int64, device="cuda")
        steps = torch.empty(B, dtype=torch.int64, device="cuda")
        ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, delta=delta, steps=steps, flags=fl)
        assert np.array_equal(col.cpu().numpy().reshape(B, n), ocol), fl
        assert np.array_equal(cost.cpu().numpy(), ocost), fl
        assert np.array_equal(types.cpu().numpy(), t_host), fl
        assert int(steps.sum()) == int(st[0]), fl
        assert delta.cpu().tolist() == [s1[0] - s0[0], s1[1] - s0[1]], fl
        assert ctx.error_flags() == 0


def test_full_round_properties(sh, ctx, full_data):
    """BASELINE config 2 at full size (3730 disjoint n=256 blocks): size-
    independent invariants + exact agreement of delta with a full rescore,
    and a random 64-block spot check against the oracle."""
    mode, n = 0, 256
    _, _, _, nb = ctx.geometry(mode, n)
    assert nb == 3730
    rows = ctx.sample_blocks(mode, n, nb, 9, 0)
    types = ctx.upload_types(full_data.types)
    cost = torch.empty(nb, dtype=torch.int64, device="cuda")
    col = torch.empty(nb * n, dtype=torch.int32, device="cuda")
    delta = torch.zeros(2, dtype=torch.int64, device="cuda")
    s0 = ctx.score_sums(types)
    ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, delta=delta)
    s1 = ctx.score_sums(types)
    assert ctx.error_flags() == 0
    t1 = types.cpu().numpy()
    # gift multiset conserved, families untouched, every block a permutation
    assert np.array_equal(np.bincount(t1, minlength=1000), np.bincount(full_data.types, minlength=1000))
    tri, tw = full_data.families
    assert np.array_equal(t1[:tri + tw], full_data.types[:tri + tw])
    c = col.cpu().numpy().reshape(nb, n)
    assert (np.sort(c, axis=1) == np.arange(n)).all()
    assert delta.cpu().tolist() == [s1[0] - s0[0], s1[1] - s0[1]]
    assert s1[2] == 0 and s1[3] == 0
    # spot-check blocks against the oracle from the same starting state
    r = rows.cpu().numpy().reshape(nb, n)
    pick = np.random.default_rng(0).choice(nb, 48, replace=False)
    t_host = full_data.types.copy()
    ocol, ocost = oracle.round_blocks(mode, full_data.wish, t_host, r[pick], ng=full_data.ng)
    assert np.array_equal(c[pick], ocol)
    assert np.array_equal(cost.cpu().numpy()[pick], ocost)
    assert np.array_equal(t1[r[pick].reshape(-1)], t_host[r[pick].reshape(-1)])


def _oracle_round_threaded(mode, wish, t_host, r, ng, threads=16):
    """oracle.round_blocks over every block of a round, split over threads
    (ctypes releases the GIL; the blocks are disjoint, so the threads apply
    their swaps to the one host type vector without conflicts)."""
    import concurrent.futures as cf
    B = r.shape[0]
    col = np.zeros(r.shape, dtype=np.int64)
    cost = np.zeros(B, dtype=np.int64)
    steps = np.zeros(B, dtype=np.uint64)
    chunk = (B + threads - 1) // threads

    def work(b0):
        b1 = min(B, b0 + chunk)
        st = np.zeros(2, dtype=np.uint64)
        c, k = oracle.round_blocks(mode, wish, t_host, r[b0:b1], stats=st, ng=ng)
        col[b0:b1], cost[b0:b1] = c, k
        return int(st[0])

    with cf.ThreadPoolExecutor(threads) as ex:
        total_steps = sum(ex.map(work, range(0, B, chunk)))
    return col, cost, total_steps


@pytest.mark.parametrize("mode,pinned,rounds", [(0, (1, 10, 19), 20), (1, (0, 10), 11)])
def test_bench_rounds_vs_oracle(sh, ctx, full_data, mode, pinned, rounds):
    """The rounds bench.py times, pinned to the oracle on the path bench.py
    runs: bench seed 2017, full rounds (3730 singles blocks on the default
    dispatch: the fused santa_sp3_kernel<.., FUSED = true>, which samples
    nothing itself but builds its register tile in-kernel from the packed
    wishlists and solves in 32-bit lattice keys; 78 twins blocks on
    santa_block_kernel<1, 1>), the reference's loop (run_rounds) with its
    default delta round sums.  The engine under test is GPUEngine itself: its
    solve_blocks runs (ctx.solve_round: the round's undo record written by the
    block kernels, the next round's rows sampled by them into the ring of
    three buffers, the delta published to the host mailbox by the round's last
    launch); the wrapper only reads the state around it.
      * pinned rounds: ALL blocks' col and exact cost (a separate
        SH_FLAG_NO_APPLY solve from the saved pre-round state), the steps, and
        the whole post-round type vector equal the oracle solving the same
        pre-round state;
      * every other round: a random sample of 64 blocks (col, cost, their new
        types) equals the oracle, and the whole post-round vector equals the
        pre-round one with the NO_APPLY solve's assignment applied;
      * every round: the rows are the host sampler's (seed, round) blocks, and
        the (S_child, S_gift) the loop reports (start sums + the block deltas,
        read through the mailbox) equal the oracle's rescore of the round's
        post-round state (mpi_single.py:151-157, mpi_twins.py:157-169)."""
    from santa_hip import _lib
    from santa_hip import sampler as S
    from santa_hip.driver import GPUEngine, World, run_rounds
    n = 256
    lo, count, stride, nb = ctx.geometry(mode, n)
    assert ctx.solve_design(mode, n, nb) == (_lib.SH_DESIGN_SPARSE3 if mode == 0 else _lib.SH_DESIGN_TWINS)
    checked, sampled, post, fused = [], [], [], []

    class Pin(GPUEngine):
        calls = 0

        def solve_blocks(self, mode_, rows_, n_, types_, delta=None, steps=None):
            k = self.calls
            self.calls += 1
            B = rows_.numel() // n_
            fused.append(self._cur is not None and self._cur[6])  # (rows sampled by the last round's kernels)
            pre = types_.cpu().numpy()
            r = rows_.cpu().numpy().reshape(B, n_)
            assert np.array_equal(r, S.sample_blocks(2017, k, lo, count, stride, n_, B)), k
            col = torch.empty(B * n_, dtype=torch.int32, device="cuda")
            cost = torch.empty(B, dtype=torch.int64, device="cuda")
            ctx.solve_blocks(mode_, rows_, n_, types_, col=col, cost=cost, flags=_lib.SH_FLAG_NO_APPLY)
            assert np.array_equal(types_.cpu().numpy(), pre), k
            st = torch.empty(B, dtype=torch.int64, device="cuda") if k in pinned else steps
            super().solve_blocks(mode_, rows_, n_, types_, delta=delta, steps=st)
            got = types_.cpu().numpy()
            c = col.cpu().numpy().reshape(B, n_)
            t_host = pre.copy()
            if k not in pinned:
                pick = np.sort(np.random.default_rng(1000 + k).choice(B, min(64, B), replace=False))
                ocol, ocost, _ = _oracle_round_threaded(mode_, full_data.wish, t_host, r[pick],
                                                        full_data.ng)
                assert np.array_equal(c[pick], ocol), k
                assert np.array_equal(cost.cpu().numpy()[pick], ocost), k
                kids = np.concatenate([r[pick].reshape(-1) + m for m in range(mode_ + 1)])
                assert np.array_equal(got[kids], t_host[kids]), k
                # the applied round = the pre-round state permuted by the NO_APPLY assignment
                want = pre.copy()
                for m in range(mode_ + 1):  # (a unit's members share its first member's type)
                    want[r + m] = pre[np.take_along_axis(r, c, axis=1)]
                assert np.array_equal(got, want), k
                sampled.append(k)
                return
            ocol, ocost, osteps = _oracle_round_threaded(mode_, full_data.wish, t_host, r, full_data.ng)
            assert np.array_equal(c, ocol), k
            assert np.array_equal(cost.cpu().numpy(), ocost), k
            assert np.array_equal(got, t_host), k
            assert int(st.sum()) == osteps, k
            checked.append(k)

        def delta_begin(self, t, d, full, after=None, **kw):
            # the round's post-round state (before a keep-if-improved rollback)
            post.append(oracle.score_sums(full_data.wish, full_data.goodkids, t.cpu().numpy())[:2])
            return super().delta_begin(t, d, full, after, **kw)

        def score_sums(self, t):
            s = super().score_sums(t)
            assert s == oracle.score_sums(full_data.wish, full_data.goodkids, t.cpu().numpy())
            return s

    reported = []
    types = ctx.upload_types(full_data.types)
    res = run_rounds(Pin(ctx), types, mode=mode, n=n, seed=2017, max_rounds=rounds, patience=1 << 30,
                     world=World(), on_round=lambda st: reported.append((st.s_child, st.s_gift)))
    assert checked == list(pinned) and res.rounds == rounds
    assert sorted(checked + sampled) == list(range(rounds))
    assert len(post) == rounds and reported == post
    # every round after the first took its rows from the previous round's block kernels
    assert fused == [False] + [True] * (rounds - 1)
    assert ctx.error_flags() == 0


def test_twins_rejected_rounds_vs_oracle(sh, ctx, full_data):
    """Keep-if-improved rounds with rollbacks (mpi_twins.py:133,166-175) on
    the path the loop runs: 12 full 78-block twins rounds, rounds 1, 4, 5 and
    9 forced to be rejected (their score is hidden from the loop by a
    score_from_sums hook, so their update must be undone).
      * serial loop, GPUEngine (undo records written by the block kernels,
        rows sampled ahead by them, mailbox sums): every round's pre-state
        equals the oracle's accepted state -- so every rollback restored it --
        and every post-round state equals the oracle solving that pre-state;
      * pipelined loop (speculative round undone and re-run after a
        rejection) and an engine without undo records (whole-state copies)
        give the same history and final state."""
    from santa_hip.driver import GPUEngine, World, run_rounds
    n, rounds, reject = 256, 12, {1, 4, 5, 9}
    lo, count, stride, nb = ctx.geometry(1, n)
    expected = [full_data.types.copy()]
    pending = []

    def hooked(base):
        class E(base):
            calls = 0

            def score_from_sums(self, sc, sg):
                k = self.calls
                self.calls += 1
                s = super().score_from_sums(sc, sg)
                return float("-inf") if k - 1 in reject else s  # (call 0 is the start score)
        return E

    class Oracle(hooked(GPUEngine)):
        def solve_blocks(self, mode_, rows_, n_, types_, delta=None, steps=None):
            B = rows_.numel() // n_
            pre = types_.cpu().numpy()
            assert np.array_equal(pre, expected[-1]), len(pending)
            super().solve_blocks(mode_, rows_, n_, types_, delta=delta, steps=steps)
            t_host = pre.copy()
            _oracle_round_threaded(mode_, full_data.wish, t_host, rows_.cpu().numpy().reshape(B, n_),
                                   full_data.ng)
            assert np.array_equal(types_.cpu().numpy(), t_host), len(pending)
            pending.append(t_host)

    def on_round(st):
        if st.accepted:
            expected.append(pending[-1])

    class Copies(hooked(GPUEngine)):
        sample_round = None

    out = []
    for eng, pipeline in ((Oracle, False), (hooked(GPUEngine), True), (Copies, False), (Copies, True)):
        types = ctx.upload_types(full_data.types)
        res = run_rounds(eng(ctx), types, mode=1, n=n, seed=31, max_rounds=rounds, patience=1 << 30,
                         world=World(), pipeline=pipeline,
                         on_round=on_round if eng is Oracle else None)
        torch.cuda.synchronize()
        hist = [(st.round, st.s_child, st.s_gift, st.accepted) for st in res.history]
        out.append((types.cpu().numpy(), hist))
    kept = [h[3] for h in out[0][1]]
    assert len(pending) == rounds and len(expected) == 1 + sum(kept)
    assert not any(kept[r] for r in reject) and sum(kept) >= 4
    assert np.array_equal(out[0][0], expected[-1])
    for t, h in out[1:]:
        assert np.array_equal(t, out[0][0]) and h == out[0][1]
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("mode,n", [(0, 2000), (1, 3000)])
def test_full_round_reference_block_sizes(sh, ctx, full_data, mode, n):
    """A full round at the reference's default block sizes (477 blocks of 2000
    singles, mpi_single.py:238-240; 6 blocks of 3000 pairs,
    mpi_twins.py:244-246): invariants, delta = rescore, and blocks spot-checked
    against the oracle."""
    _, _, _, nb = ctx.geometry(mode, n)
    assert nb == (477 if mode == 0 else 6)
    rows = ctx.sample_blocks(mode, n, nb, 4, 0)
    types = ctx.upload_types(full_data.types)
    cost = torch.empty(nb, dtype=torch.int64, device="cuda")
    col = torch.empty(nb * n, dtype=torch.int32, device="cuda")
    delta = torch.zeros(2, dtype=torch.int64, device="cuda")
    s0 = ctx.score_sums(types)
    ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, delta=delta)
    s1 = ctx.score_sums(types)
    assert ctx.error_flags() == 0
    t1 = types.cpu().numpy()
    assert np.array_equal(np.bincount(t1, minlength=1000), np.bincount(full_data.types, minlength=1000))
    c = col.cpu().numpy().reshape(nb, n)
    assert (np.sort(c, axis=1) == np.arange(n)).all()
    assert delta.cpu().tolist() == [s1[0] - s0[0], s1[1] - s0[1]]
    assert s1[2] == 0 and s1[3] == 0
    r = rows.cpu().numpy().reshape(nb, n)
    pick = np.random.default_rng(1).choice(nb, 2, replace=False)
    t_host = full_data.types.copy()
    ocol, ocost = oracle.round_blocks(mode, full_data.wish, t_host, r[pick], ng=full_data.ng)
    assert np.array_equal(c[pick], ocol)
    assert np.array_equal(cost.cpu().numpy()[pick], ocost)


@pytest.mark.parametrize("n", [300, 700, 1100, 2000])
def test_large_block_wave_configs_agree(sh, ctx, full_data, n):
    """The row-rebuild kernel runs 8 waves per block when a launch has at
    least one block per CU and 16 otherwise: 260 blocks in one launch equal
    the same blocks in launches of 65 (col, cost, steps, deltas, the new
    types), and equal the staged-row lattice kernel's one launch (the
    default); two of them equal the oracle."""
    from santa_hip import _lib
    B = 260
    rows = ctx.sample_blocks(0, n, B, 11, 3)
    outs = []
    for chunk, fl in ((B, _lib.SH_FLAG_BIG_ROWS), (65, _lib.SH_FLAG_BIG_ROWS), (B, 0)):
        types = ctx.upload_types(full_data.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        steps = torch.empty(B, dtype=torch.int64, device="cuda")
        delta = torch.zeros(2, dtype=torch.int64, device="cuda")
        for b0 in range(0, B, chunk):
            sl = slice(b0 * n, (b0 + chunk) * n)
            d = torch.zeros(2, dtype=torch.int64, device="cuda")
            ctx.solve_blocks(0, rows[sl], n, types, col=col[sl], cost=cost[b0:b0 + chunk],
                             steps=steps[b0:b0 + chunk], delta=d, flags=fl)
            delta += d
        outs.append([x.cpu().numpy() for x in (col, cost, steps, delta, types)])
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert np.array_equal(x, y), n
    assert ctx.error_flags() == 0
    r = rows.cpu().numpy().reshape(B, n)
    t_host = full_data.types.copy()
    ocol, ocost = oracle.round_blocks(0, full_data.wish, t_host, r[[5, 201]], ng=full_data.ng)
    assert np.array_equal(outs[0][0].reshape(B, n)[[5, 201]], ocol)
    assert np.array_equal(outs[0][1][[5, 201]], ocost)


# --------------------------------------------------------------------------- score
def test_score_matches_golden(sh, ctx, full_data):
    g = golden_json("santa_score.json")
    base = g["entries"][0]
    types = ctx.upload_types(full_data.types)
    assert ctx.score_sums(types) == (base["S_child"], base["S_gift"], 0, 0)
    assert ctx.score(types) == base["score"]
    # a perturbed state vs the oracle, with broken families reported
    t2 = full_data.types.copy()
    rng = np.random.default_rng(1)
    idx = rng.choice(full_data.nc, 5000, replace=False)
    t2[idx] = rng.integers(0, 1000, 5000)
    got = ctx.score_sums(ctx.upload_types(t2))
    want = oracle.score_sums(full_data.wish, full_data.goodkids, t2)
    assert got == want
    assert want[2] + want[3] > 0
    with pytest.raises(AssertionError):
        ctx.score(ctx.upload_types(t2))


def test_avg_normalized_happiness_api(sh, full_data):
    g = golden_json("santa_score.json")
    s = sh.avg_normalized_happiness(full_data.pred(), full_data.goodkids, full_data.wish)
    assert s == g["entries"][0]["score"]


# --------------------------------------------------------------------------- driver
@pytest.mark.parametrize("check", [0, None])
@pytest.mark.parametrize("mode", ["single", "twins"])
def test_trajectory_gpu_matches_reference(sh, ctx, full_data, mode, check, tmp_path):
    """The reference's my_optimizer (3 rounds, P blocks per round) replayed
    on the GPU: scores, states and the per-round checkpoint CSV (byte-
    identical to the reference's to_csv, mpi_single.py:177) all equal; with
    the reference's full rescore every round (check = 0, the rescored states'
    digests compared too) and with the default delta sums (check = None)."""
    import hashlib

    from santa_hip import data as D
    from santa_hip.driver import GPUEngine, World, run_rounds
    g = golden_json(f"trajectory_{mode}.json")
    types = ctx.upload_types(full_data.types)
    shas = []
    csvs = []

    class Rec(GPUEngine):
        def score_sums(self, t):
            shas.append(sha(t.cpu().numpy()))
            return super().score_sums(t)

    def checkpoint(st):
        p = tmp_path / f"r{st.round}.csv"
        D.write_submission(str(p), types.cpu().numpy())
        data = open(p, "rb").read()
        csvs.append({"sha256": hashlib.sha256(data).hexdigest(), "bytes": len(data)})

    m = 0 if mode == "single" else 1
    res = run_rounds(Rec(ctx), types, mode=m, n=g["n"], blocks_per_round=g["P"], seed=g["seed"],
                     max_rounds=g["rounds"], world=World(), score0=g["score0"], on_round=checkpoint,
                     score_check_every=check)
    assert [st.score for st in res.history] == [r["score"] for r in g["per_round"]]
    assert csvs == [r["csv"] for r in g["per_round"]]
    if check == 0:
        assert shas == [r["types_sha"] for r in g["per_round"]]


def test_optimize_block_api(sh, full_data, santa_blocks):
    from santa_hip import data as D
    z, meta = santa_blocks
    sh.init(full_data.wish, full_data.goodkids)
    slots = D.slot_ids(full_data.types, full_data.nq)
    import pandas as pd
    subm = pd.DataFrame({"ChildId": np.arange(full_data.nc), "GiftId": full_data.types.astype(np.int64)})
    for m in meta[:3] + [x for x in meta if x["mode"] == "twins"][:2]:
        k = m["i"]
        blk = z[f"rows{k}"].astype(np.int64)
        if m["mode"] == "single":
            cids, gids = sh.optimize_block(blk, slots)
            assert np.array_equal(gids, slots[blk][z[f"col{k}"]])
        else:
            cids, gids = sh.optimize_block_twins(blk, subm)
            assert np.array_equal(gids, full_data.types[blk][z[f"col{k}"]].astype(np.int64))
        assert np.array_equal(cids, blk)


# --------------------------------------------------------------------------- errors
def test_error_paths(sh, ctx, full_data):
    types = ctx.upload_types(full_data.types)
    bad = torch.full((256,), full_data.nc + 5, dtype=torch.int32, device="cuda")
    ctx.solve_blocks(0, bad, 256, types)
    assert ctx.error_flags() & 1
    assert np.array_equal(types.cpu().numpy(), full_data.types)  # skipped block wrote nothing
    with pytest.raises(ValueError):
        ctx.solve_blocks(0, torch.zeros(5000, dtype=torch.int32, device="cuda"), 5000, types)
    with pytest.raises(ValueError):  # one past SH_MAX_N_SANTA
        ctx.solve_blocks(0, torch.zeros(4097, dtype=torch.int32, device="cuda"), 4097, types)
    with pytest.raises(ValueError):
        ctx.sample_blocks(0, 256, 5000, 1, 0)
    with pytest.raises(ValueError):
        sh.linear_sum_assignment(np.array([[np.nan, 0.0], [0.0, 0.0]]))


def test_pack_unpack_roundtrip(sh, ctx, full_data):
    types = ctx.upload_types(full_data.types)
    rows = ctx.sample_blocks(1, 64, 10, 3, 3)
    buf = torch.empty(rows.numel(), dtype=torch.int16, device="cuda")
    ctx.pack_types(types, rows, buf)
    assert np.array_equal(buf.cpu().numpy(), full_data.types[rows.cpu().numpy()])
    t2 = torch.zeros_like(types)
    ctx.unpack_types(t2, rows, buf, 1)
    r = rows.cpu().numpy()
    t2n = t2.cpu().numpy()
    assert np.array_equal(t2n[r], full_data.types[r]) and np.array_equal(t2n[r + 1], full_data.types[r])
    # triplet units: all three members take the unit's value
    rows3 = ctx.sample_blocks(2, 64, 5, 3, 3)
    buf3 = torch.empty(rows3.numel(), dtype=torch.int16, device="cuda")
    ctx.pack_types(types, rows3, buf3)
    t3 = torch.zeros_like(types)
    ctx.unpack_types(t3, rows3, buf3, 2)
    r3 = rows3.cpu().numpy()
    t3n = t3.cpu().numpy()
    for m in range(3):
        assert np.array_equal(t3n[r3 + m], full_data.types[r3])


# --------------------------------------------------------------------------- argmin paths
def test_fast_and_exact_argmin_agree(sh, ctx, full_data):
    """The packed-key DPP argmin and the two-pass exact argmin (forced by
    SH_FLAG_EXACT_ARGMIN) make identical decisions; on the sparse design
    (SH_FLAG_SP_TILE) the flag sends every block to the fallback launch's
    windowed-key solver with the exact argmin."""
    from santa_hip import _lib
    for mode, n, B in ((0, 256, 32), (1, 256, 4)):
        rows = ctx.sample_blocks(mode, n, B, 31, 2)
        outs = []
        extra = ((_lib.SH_FLAG_SP_TILE | _lib.SH_FLAG_EXACT_ARGMIN, _lib.SH_FLAG_DT_TILE | _lib.SH_FLAG_EXACT_ARGMIN)
                 if mode == 0 else ())
        for fl in (0, _lib.SH_FLAG_EXACT_ARGMIN) + extra:
            types = ctx.upload_types(full_data.types)
            col = torch.empty(B * n, dtype=torch.int32, device="cuda")
            ctx.solve_blocks(mode, rows, n, types, col=col, flags=fl)
            outs.append((col.cpu().numpy(), types.cpu().numpy()))
        for o in outs[1:]:
            assert np.array_equal(outs[0][0], o[0])
            assert np.array_equal(outs[0][1], o[1])


def test_lsap_wide_range_int64_uses_exact_fallback(sh):
    """Spreads beyond the packed key's 2^52 window take the exact argmin."""
    rng = np.random.default_rng(11)
    C = rng.integers(-(1 << 49), 1 << 49, size=(3, 128, 128), dtype=np.int64)
    col, cost = sh.solve_batched(torch.from_numpy(C).cuda())
    ocol, ocost = oracle.lsap_i64_batched(C)
    assert np.array_equal(col.cpu().numpy(), ocol)
    assert np.array_equal(cost.cpu().numpy(), ocost)
    with pytest.raises(ValueError):
        sh.solve_batched(torch.from_numpy(C * 4).cuda())


@pytest.mark.parametrize("maximize", [False, True])
def test_lsap_int64_min_takes_float_path(sh, maximize):
    """An int64 entry at INT64_MIN (np.abs and negation wrap there) is out of
    the exact-int64 range: linear_sum_assignment replays scipy's float64
    arithmetic instead, for minimise and maximise alike."""
    rng = np.random.default_rng(3)
    C = rng.integers(-50, 50, size=(9, 9), dtype=np.int64)
    C[2, 5] = np.iinfo(np.int64).min
    _, got = sh.linear_sum_assignment(C, maximize=maximize)
    Cf = C.astype(np.float64)
    _, want = oracle.lsap(-Cf if maximize else Cf)
    assert np.array_equal(got, want)
    with pytest.raises(ValueError):
        sh.solve_batched(torch.from_numpy(C[None]).cuda())


def test_no_fallback_on_santa_rounds(sh, ctx, full_data):
    """Santa cost spreads stay inside the packed key's window: the exact
    two-pass argmin is never needed on real rounds (performance guard)."""
    ctx.fallback_steps()
    types = ctx.upload_types(full_data.types)
    for mode, n in ((0, 256), (1, 256)):
        _, _, _, nb = ctx.geometry(mode, n)
        rows = ctx.sample_blocks(mode, n, min(nb, 512), 5, 0)
        ctx.solve_blocks(mode, rows, n, types)
    assert ctx.fallback_steps() == 0


def _round_outputs(ctx, full_data, mode, rows, nn, B, fl=0):
    types = ctx.upload_types(full_data.types)
    col = torch.empty(B * nn, dtype=torch.int32, device="cuda")
    cost = torch.empty(B, dtype=torch.int64, device="cuda")
    delta = torch.zeros(2, dtype=torch.int64, device="cuda")
    steps = torch.empty(B, dtype=torch.int64, device="cuda")
    ctx.solve_blocks(mode, rows, nn, types, col=col, cost=cost, delta=delta, steps=steps, flags=fl)
    return [x.cpu().numpy() for x in (col, cost, delta, steps, types)]


@pytest.mark.parametrize("design", ["tile2", "sp1"])
def test_sparse_overflow_fallback(sh, ctx, full_data, design):
    """Blocks that do not fit the sparse kernels' on-chip capacity (sp1: the
    LDS hit-list budget; tile2: the overflow list of rows with more than 32
    hits, capacity budget / 16 entries) are solved by the register-tile
    fallback launch; any budget gives the same round (all blocks
    overflowing, some, none), repeated calls included (the double-buffered
    overflow counters)."""
    from santa_hip import _lib
    B, nn = 96, 256
    rows = ctx.sample_blocks(0, nn, B, 5, 3)
    want = _round_outputs(ctx, full_data, 0, rows, nn, B, _lib.SH_FLAG_VT_TILE)
    fl = {"tile2": _lib.SH_FLAG_SP_TILE, "sp1": _lib.SH_FLAG_SP1}[design]
    budgets = (16, 1600, 2400, 0, 0, 800, 0) if design != "sp1" else (6000, 16500, 17500, 0, 0, 4096, 0)
    try:
        for budget in budgets:
            cap = ctx.set_sparse_budget(budget)
            assert cap >= 0
            got = _round_outputs(ctx, full_data, 0, rows, nn, B, fl)
            for x, y in zip(want, got):
                assert np.array_equal(x, y), budget
        assert ctx.error_flags() == 0
    finally:
        ctx.set_sparse_budget(0)


def test_kernel_designs_agree(sh, ctx, full_data):
    """The one-wave sparse-tile kernel (SH_FLAG_SP_TILE), the default dispatch, the 4-wave
    register-tile kernel (SH_FLAG_VT_TILE), the 4-wave LDS-tile kernel
    (SH_FLAG_LDS_TILE) and the dense-tile one-wave kernel (SH_FLAG_DT_TILE)
    produce identical rounds: col, cost, deltas, steps, state.  The retired one-wave register kernel's flag is refused."""
    from santa_hip import _lib
    mode = 0
    for B, nn in ((64, 256), (16, 100), (8, 37), (8, 130), (4, 1), (6, 255), (5, 64)):
        rows = ctx.sample_blocks(mode, nn, B, 77, 9)
        outs = []
        for fl in (_lib.SH_FLAG_SP_TILE, 0, _lib.SH_FLAG_SP1, _lib.SH_FLAG_VT_TILE, _lib.SH_FLAG_LDS_TILE,
                   _lib.SH_FLAG_DT_TILE):
            types = ctx.upload_types(full_data.types)
            col = torch.empty(B * nn, dtype=torch.int32, device="cuda")
            cost = torch.empty(B, dtype=torch.int64, device="cuda")
            delta = torch.zeros(2, dtype=torch.int64, device="cuda")
            steps = torch.empty(B, dtype=torch.int64, device="cuda")
            ctx.solve_blocks(mode, rows, nn, types, col=col, cost=cost, delta=delta, steps=steps,
                             flags=fl)
            outs.append([x.cpu().numpy() for x in (col, cost, delta, steps, types)])
        for other in outs[1:]:
            for x, y in zip(outs[0], other):
                assert np.array_equal(x, y), (B, nn)
    types = ctx.upload_types(full_data.types)
    with pytest.raises(ValueError, match="retired"):
        ctx.solve_blocks(mode, ctx.sample_blocks(mode, 256, 4, 1, 0), 256, types, flags=_lib.SH_FLAG_SW_TILE)
    with pytest.raises(ValueError, match="retired"):
        ctx.solve_design(mode, 256, 4, _lib.SH_FLAG_SW_TILE)
    # round 2's 64-bit-key one-wave kernel (santa_sp2_kernel) left the library too
    with pytest.raises(ValueError, match="retired"):
        ctx.solve_blocks(mode, ctx.sample_blocks(mode, 256, 4, 1, 0), 256, types, flags=_lib.SH_FLAG_SP2)
    with pytest.raises(ValueError, match="retired"):
        ctx.solve_design(mode, 256, 3730, _lib.SH_FLAG_SP2)


def test_shard_designs_agree(sh, ctx, full_data):
    """One GPU's shard of a round at 4 and 8 GPUs (933 / 466 blocks: the
    sparse and the dense-tile kernels by default) equals the sparse kernel's
    result, also with every block sent through the windowed-key re-solve
    (SH_FLAG_TEST_RANGE) and the exact argmin, and on the dense-tile, 4-wave
    register-tile and 4-wave LDS-tile kernels."""
    from santa_hip import _lib
    for B in (933, 466):
        rows = ctx.sample_blocks(0, 256, B, 2017, 0)
        outs = []
        for fl in (_lib.SH_FLAG_SP_TILE, 0, _lib.SH_FLAG_TEST_RANGE, _lib.SH_FLAG_EXACT_ARGMIN, _lib.SH_FLAG_DT_TILE,
                   _lib.SH_FLAG_VT_TILE, _lib.SH_FLAG_LDS_TILE):
            types = ctx.upload_types(full_data.types)
            col = torch.empty(B * 256, dtype=torch.int32, device="cuda")
            cost = torch.empty(B, dtype=torch.int64, device="cuda")
            delta = torch.zeros(2, dtype=torch.int64, device="cuda")
            steps = torch.empty(B, dtype=torch.int64, device="cuda")
            ctx.solve_blocks(0, rows, 256, types, col=col, cost=cost, delta=delta, steps=steps, flags=fl)
            outs.append([x.cpu().numpy() for x in (col, cost, delta, steps, types)])
        for other in outs[1:]:
            for x, y in zip(outs[0], other):
                assert np.array_equal(x, y), B
    assert ctx.error_flags() == 0


def test_design_dispatch(sh, ctx):
    """Singles n=256: the sparse kernel for a full round (3730 blocks) and for
    the shards at 2 and 4 GPUs (1865, 933), the dense-tile one-wave kernel
    when the launch fits in one resident wave of its blocks (one GPU's shard
    at 8 GPUs: 466), the sparse kernel again when forced; twins and large
    blocks have one default design each."""
    from santa_hip import _lib
    assert ctx.solve_design(0, 256, 3730) == _lib.SH_DESIGN_SPARSE3
    assert ctx.solve_design(0, 256, 466) == _lib.SH_DESIGN_DT_TILE
    assert ctx.resident_blocks(0, 256, 466) >= 466
    assert ctx.solve_design(0, 256, 466, _lib.SH_FLAG_SP_TILE) == _lib.SH_DESIGN_SPARSE3
    assert ctx.solve_design(0, 256, 3730, _lib.SH_FLAG_DT_TILE) == _lib.SH_DESIGN_DT_TILE
    assert ctx.resident_blocks(0, 256, 466, _lib.SH_FLAG_DT_TILE) >= 466
    assert ctx.solve_design(0, 256, 3730, _lib.SH_FLAG_SP1) == 0
    assert ctx.solve_design(0, 256, 933) == _lib.SH_DESIGN_SPARSE3
    assert ctx.solve_design(0, 256, 933, _lib.SH_FLAG_VT_TILE) == 3
    assert ctx.resident_blocks(0, 256, 933) >= 933
    assert ctx.solve_design(0, 256, 1865) == _lib.SH_DESIGN_SPARSE3
    # the register-tile design holds a whole round at once (4 waves per SIMD)
    assert ctx.resident_blocks(0, 256, 3730) >= 3730
    assert ctx.solve_design(1, 256, 78) == 4
    assert ctx.solve_design(0, 2000, 477) == _lib.SH_DESIGN_LARGE_LB
    assert ctx.solve_design(0, 2000, 1) == _lib.SH_DESIGN_LARGE_LB
    assert ctx.resident_blocks(0, 2000, 477) >= 477  # (two blocks per CU: the round at once)
    assert ctx.solve_design(0, 2000, 477, _lib.SH_FLAG_BIG_ROWS) == 5
    assert ctx.solve_design(0, 4096, 1) == 5
    assert ctx.solve_design(1, 3000, 6) == 5
    assert ctx.solve_design(2, 256, 6) == 5


# --------------------------------------------------------------------------- RCCL exchange
def test_exchange_over_rccl(sh, ctx, full_data):
    """The per-round exchange (pack -> all-gather -> unpack) and the N>1
    round loop through a real RCCL process group (one rank: this box has one
    GPU; the N>1 logic is covered by the gloo tests).  Catches dtypes RCCL
    does not carry and stream-ordering faults of the async delta all-reduce."""
    import socket

    import torch.distributed as dist
    from santa_hip.driver import GPUEngine, World, exchange, run_rounds
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        for mode, n in ((0, 256), (1, 64)):
            _, _, _, nb = ctx.geometry(mode, n)
            rows = ctx.sample_blocks(mode, n, nb, 7, 1)
            types = ctx.upload_types(full_data.types)
            ctx.solve_blocks(mode, rows, n, types)
            want = types.clone()
            bufs = {}
            exchange(GPUEngine(ctx), World(0, 1, None), mode, rows, n, nb, types, bufs)
            torch.cuda.synchronize()
            # the all-gathered bytes are this rank's packed new types
            assert torch.equal(bufs["recv"][:rows.numel()], want[rows.long()]), mode
            assert torch.equal(types, want), mode

        # the whole N > 1 round loop over this RCCL group: exchange, the delta
        # all-reduce issued async and waited by the side stream, the error-flag
        # agreement; same history and state as the one-rank loop
        class RcclWorld(World):
            @property
            def distributed(self) -> bool:
                return True

        out = []
        for w in (World(), RcclWorld(0, 1, None)):
            types = ctx.upload_types(full_data.types)
            res = run_rounds(GPUEngine(ctx), types, mode=0, n=256, seed=3, max_rounds=5, patience=1 << 30,
                             world=w, pipeline=True, score_check_every=2)
            torch.cuda.synchronize()
            out.append((types.cpu().numpy(), [(st.s_child, st.s_gift, st.score) for st in res.history]))
        assert np.array_equal(out[0][0], out[1][0]) and out[0][1] == out[1][1]
    finally:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- edge sizes
@pytest.mark.parametrize("n,B,picks", [(100, 4096, (0, 1, 4095)), (128, 8192, (7, 8191)),
                                      (256, 65536, (0, 65535))])
def test_lsap_large_batch_configs_vs_oracle(sh, n, B, picks):
    """Large batches run one wave per instance with several columns per
    thread (n <= 128 from 4096 instances, n = 256 from 65536): instances of
    the device-generated stream equal the oracle on the host mirror of the
    hash, permutation and cost."""
    from santa_hip import lsap as L
    from santa_hip.sampler import hash_matrix
    col, cost = L.solve_hash(5, 1 << 16, n, B, device=0)
    c = col.cpu().numpy().reshape(B, n)
    for b in picks:
        C = hash_matrix(5, b, n, 1 << 16).astype(np.int64)[None]
        ocol, ocost = oracle.lsap_i64_batched(C)
        assert np.array_equal(c[b], ocol[0]), (n, B, b)
        assert int(cost.cpu()[b]) == int(ocost[0]), (n, B, b)


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 255])
def test_lsap_edge_sizes_vs_oracle(sh, n):
    """Wave-boundary and degenerate sizes (one lane, partial waves, one column
    past a wave) through the batched solver, against the oracle; ties
    included (small modulus)."""
    rng = np.random.default_rng(1000 + n)
    for mod in (3, 1 << 16):
        C = rng.integers(0, mod, size=(3, n, n), dtype=np.int64)
        col, cost = sh.solve_batched(torch.from_numpy(C).cuda())
        ocol, ocost = oracle.lsap_i64_batched(C)
        assert np.array_equal(col.cpu().numpy(), ocol), (n, mod)
        assert np.array_equal(cost.cpu().numpy(), ocost), (n, mod)


def test_empty_batches_are_noops(sh, ctx, full_data):
    """B = 0 (an empty shard, e.g. a rank with no blocks) is accepted and
    changes nothing, like scipy on an empty problem list."""
    col, cost = sh.solve_batched(torch.empty((0, 8, 8), dtype=torch.int64, device="cuda"))
    assert col.shape == (0, 8) and cost.shape == (0,)
    types = ctx.upload_types(full_data.types)
    ctx.solve_blocks(0, torch.empty(0, dtype=torch.int32, device="cuda"), 256, types)
    torch.cuda.synchronize()
    assert np.array_equal(types.cpu().numpy(), full_data.types)
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("mode,n,B", [(0, 1, 5), (0, 2, 7), (0, 63, 3), (0, 65, 3),
                                      (1, 1, 4), (1, 2, 3), (1, 65, 2),
                                      (2, 1, 4), (2, 2, 3), (2, 65, 2)])
def test_santa_edge_block_sizes_vs_oracle(sh, ctx, full_data, mode, n, B):
    """Santa blocks of degenerate / wave-boundary sizes: the fused kernels
    equal the oracle (col, cost, whole type vector, deltas)."""
    from santa_hip import _lib
    rows = ctx.sample_blocks(mode, n, B, 77, 2)
    t_host = full_data.types.copy()
    ocol, ocost = oracle.round_blocks(mode, full_data.wish, t_host, rows.cpu().numpy().reshape(B, n),
                                      ng=full_data.ng)
    s0 = oracle.score_sums(full_data.wish, full_data.goodkids, full_data.types)
    s1 = oracle.score_sums(full_data.wish, full_data.goodkids, t_host)
    for fl in ((0, _lib.SH_FLAG_SP_TILE, _lib.SH_FLAG_SP1, _lib.SH_FLAG_DT_TILE) if mode == 0 else (0,)):
        types = ctx.upload_types(full_data.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        delta = torch.zeros(2, dtype=torch.int64, device="cuda")
        ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, delta=delta, flags=fl)
        assert np.array_equal(col.cpu().numpy().reshape(B, n), ocol), fl
        assert np.array_equal(cost.cpu().numpy(), ocost), fl
        assert np.array_equal(types.cpu().numpy(), t_host), fl
        assert delta.cpu().tolist() == [s1[0] - s0[0], s1[1] - s0[1]], fl
        assert ctx.error_flags() == 0


# --------------------------------------------------------------------------- config 4 on the HIP path
@pytest.mark.parametrize("mode,rounds", [(0, 3), (1, 3), (2, 3)])
def test_two_ranks_on_the_hip_path_equal_one_rank(sh, ctx, full_data, mode, rounds):
    """Config 4's sharding + exchange through GPUEngine: two ranks (one
    process each, both on cuda:0, gloo all-gather) run full rounds (3730
    singles / 78 twin blocks) and end with the single-rank run's type vector
    and every per-round (S_child, S_gift), bit for bit."""
    import socket

    import torch.multiprocessing as mp
    from multirank_gpu import rank_main
    from santa_hip.driver import GPUEngine, World, run_rounds
    types = ctx.upload_types(full_data.types)
    sums = []

    class Rec(GPUEngine):
        def score_sums(self, t):
            s = super().score_sums(t)
            sums.append(s[:2])
            return s

    res = run_rounds(Rec(ctx), types, mode=mode, n=256, seed=41, max_rounds=rounds, patience=100,
                     world=World(), score_check_every=0)  # (the reference: a full rescore every round)
    want = types.cpu().numpy()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(rank_main, args=(2, port, mode, 256, rounds, 41, out), nprocs=2, join=True)
    for r in range(2):
        t, sm, scores, flags, full = out[r]
        assert flags == 0
        assert np.array_equal(t, want), f"rank {r} state differs"
        # two ranks take each round's sums from the delta all-reduce (§8(e));
        # they equal the one-rank run's full rescore of every round
        assert sm == sums[1:], f"rank {r} per-round sums differ"  # (sums[0]: the start state)
        assert scores == [st.score for st in res.history]
        # one rescore of the start state (the last round's check is internal);
        # a rejected last round (twins) adds the final state's check
        assert full[:1] == sums[:1] and len(full) <= 2


def test_bench_launches_n_ranks(sh):
    """`bench.py --gpus 2` started by hand launches its two ranks itself and
    reports n_gpus = 2 (here both on the one GPU of the box, over gloo), with
    the CPU baselines (timed by the launcher before the ranks start: the
    reference's round B1 and the C port) on the N > 1 line too."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--one-device", "--dist-backend", "gloo", "--cpu-seconds", "1",
                        "--b1-seconds", "1"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["blocks_per_round"] == 3730
    cb = line["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert set(cb["b1_blocks_per_s"]) and all(v > 0 for v in cb["b1_blocks_per_s"].values())
    # the whole-host comparator beside the leased-core figures
    wn = cb["whole_node"]
    assert wn["cores"] >= cb["cores"] and wn["port_blocks_per_s"] >= cb["value"]
    assert wn["b1_blocks_per_s"] > 0 and wn["kind"] == "projected"
    # rank 0's shard carries HBM traffic from a PMC summary of the same launch size, or says why not
    roof = line["roofline"]
    assert roof.get("traffic") is not None or roof.get("traffic_note"), roof


# --------------------------------------------------------------------------- input validation
@pytest.mark.parametrize("mode,n,fl", [(0, 256, 128), (0, 256, 256), (0, 256, 8), (0, 256, 32), (0, 256, 4096),
                                       (1, 256, 0), (0, 300, 0), (1, 300, 0)])
def test_gift_type_out_of_range_is_flagged_not_used(sh, ctx, full_data, mode, n, fl):
    """A current gift type outside [0, ng) in a block (it would index the
    kernels' on-chip tables) makes every kernel design skip that block and
    raise SH_ERRF_TYPE; the other blocks of the launch are solved."""
    from santa_hip import _lib
    B = 3
    rows = ctx.sample_blocks(mode, n, B, 5, 1)
    t = full_data.types.copy()
    bad_child = int(rows[n + 7])        # a child of block 1
    t[bad_child] = full_data.ng         # one past the last gift type
    if mode == 1:
        t[bad_child + 1] = full_data.ng
    types = torch.from_numpy(t).cuda()  # (bypasses upload_types' host check on purpose)
    ctx.error_flags()
    ctx.solve_blocks(mode, rows, n, types, flags=fl)
    flags = ctx.error_flags()
    assert flags & _lib.SH_ERRF_TYPE, flags
    got = types.cpu().numpy()
    r = rows.cpu().numpy().reshape(B, n)
    assert np.array_equal(got[r[1]], t[r[1]])                       # skipped whole
    t_host = full_data.types.copy()
    ocol, _ = oracle.round_blocks(mode, full_data.wish, t_host, r[[0, 2]], ng=full_data.ng)
    assert np.array_equal(got[r[[0, 2]].reshape(-1)], t_host[r[[0, 2]].reshape(-1)])
    with pytest.raises(ValueError):
        ctx.upload_types(t)


def test_context_on_a_second_device(sh, full_data):
    """A context bound to device 1 works while device 0 is current (the C-ABI
    switches to the context's device and back)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("one visible GPU")
    c1 = sh.SantaGPU.from_data(full_data, 1)
    torch.cuda.set_device(0)
    types = c1.upload_types(full_data.types)
    rows = c1.sample_blocks(0, 256, 8, 3, 0)
    c1.solve_blocks(0, rows, 256, types)
    assert torch.cuda.current_device() == 0
    t_host = full_data.types.copy()
    oracle.round_blocks(0, full_data.wish, t_host, rows.cpu().numpy().reshape(8, 256), ng=full_data.ng)
    assert np.array_equal(types.cpu().numpy(), t_host)
    assert c1.error_flags() == 0


# --------------------------------------------------------------------------- CLI end to end
@pytest.mark.parametrize("mode", ["single", "twins", "triplets"])
def test_cli_rounds_end_to_end(sh, full_data, mode, tmp_path, capsys):
    """`python -m santa_hip.driver` (the reference scripts' entry, no
    arguments there): seeded synthetic data, a few rounds, the per-round
    checkpoint and the final CSV.  The final CSV keeps every family on one
    gift and every gift type at its quantity; its score is the printed best;
    the pipelined and serial loops write byte-identical files."""
    import json

    import oracle
    from santa_hip import data as D
    from santa_hip.driver import main
    outs = []
    for extra in ([], ["--no-pipeline"]):
        p = tmp_path / f"sub_{len(outs)}.csv"
        assert main(["--mode", mode, "--block-size", "128", "--rounds", "3", "--out", str(p),
                     "--check-disjoint", "--seed", "5"] + extra) == 0
        lines = [json.loads(x) for x in capsys.readouterr().out.strip().splitlines()]
        outs.append((p.read_bytes(), lines))
    assert outs[0][0] == outs[1][0]
    assert [x.get("score") for x in outs[0][1]] == [x.get("score") for x in outs[1][1]]
    t = D.read_submission(str(tmp_path / "sub_0.csv"), full_data.nc, full_data.ng)
    assert np.array_equal(np.bincount(t, minlength=full_data.ng), np.bincount(full_data.types, minlength=full_data.ng))
    sc, sg, bt, btw = oracle.score_sums(full_data.wish, full_data.goodkids, t)
    assert bt == 0 and btw == 0
    s = oracle.score_from_sums(sc, sg, full_data.nc, full_data.ng, full_data.n_wish, full_data.n_good)
    # singles keep every round (the last round's state); twins/triplets the best one
    want = outs[0][1][-2]["score"] if mode == "single" else outs[0][1][-1]["best_score"]
    assert s == want
    # --checkpoint-every rewrites --out after each round (the reference's to_csv per round)
    p = tmp_path / "ck.csv"
    assert main(["--mode", mode, "--block-size", "128", "--rounds", "2", "--out", str(p),
                 "--checkpoint-every", "1", "--seed", "5"]) == 0
    capsys.readouterr()
    assert p.exists() and p.stat().st_size > 0


def test_no_apply_solves_overlapping_blocks(sh, ctx, full_data):
    """SH_FLAG_NO_APPLY: blocks are solved and reported (col, cost) but the
    gift types stay untouched, so overlapping blocks (the same block twice,
    blocks of two samplings) each equal the oracle's solve from the initial
    state; every design honours it."""
    from santa_hip import _lib
    n = 256
    r0 = ctx.sample_blocks(0, n, 6, 3, 0)
    r1 = ctx.sample_blocks(0, n, 6, 3, 1)
    rows = torch.cat([r0, r1, r0[:n]])  # overlapping blocks
    B = rows.numel() // n
    r = rows.cpu().numpy().reshape(B, n)
    want = []
    for b in range(B):
        C = oracle.cost_single(full_data.wish, full_data.types, r[b], ng=full_data.ng)
        _, oc = oracle.lsap(C)
        want.append((oc, int(C[np.arange(n), oc].sum())))
    for fl in (0, _lib.SH_FLAG_SP_TILE, _lib.SH_FLAG_SP1, _lib.SH_FLAG_LDS_TILE, _lib.SH_FLAG_VT_TILE,
               _lib.SH_FLAG_DT_TILE):
        types = ctx.upload_types(full_data.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        ctx.solve_blocks(0, rows, n, types, col=col, cost=cost, flags=fl | _lib.SH_FLAG_NO_APPLY)
        assert np.array_equal(types.cpu().numpy(), full_data.types), fl
        c = col.cpu().numpy().reshape(B, n)
        for b in range(B):
            assert np.array_equal(c[b], want[b][0]) and int(cost[b]) == want[b][1], (fl, b)
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("nw,ng,nq", [(10, 300, 100), (7, 200, 150), (10, 80, 375), (12, 100, 300),
                                      (104, 200, 100), (100, 120, 200)])
def test_small_wishlists_match_oracle(sh, nw, ng, nq):
    """The tile build's three wishlist loads: lengths that are not a multiple
    of 4 and odd lengths (2-byte gifts), n_wish = 104 (16-byte windows of the
    8-byte aligned rows), n_wish = 12 and 100 (the context's 10-bit packed
    rows); few gift types (types with 4+ columns in a
    block: the column-sort spill list; rows with more than 32 hits: the
    overflow list and, past its capacity, the fallback launch): the sparse
    design and the LDS-tile kernel equal the oracle's round bit for bit."""
    from santa_hip import _lib
    from santa_hip import data as D
    sd = D.synthetic(seed=5, nc=ng * nq, ng=ng, nq=nq, n_wish=nw, n_good=50)
    c = sh.SantaGPU.from_data(sd, 0)
    n = 256
    B = min(24, c.geometry(0, n)[3])
    rows = c.sample_blocks(0, n, B, 3, 0)
    r = rows.cpu().numpy().reshape(B, n)
    want_types = sd.types.copy()
    want_col, want_cost = oracle.round_blocks(0, sd.wish, want_types, r, ng=ng)
    for fl in (_lib.SH_FLAG_SP_TILE, _lib.SH_FLAG_LDS_TILE, _lib.SH_FLAG_VT_TILE, _lib.SH_FLAG_DT_TILE):
        types = c.upload_types(sd.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        c.solve_blocks(0, rows, n, types, col=col, cost=cost, flags=fl)
        assert np.array_equal(col.cpu().numpy().reshape(B, n), want_col), (nw, ng, fl)
        assert np.array_equal(cost.cpu().numpy(), want_cost), (nw, ng, fl)
        assert np.array_equal(types.cpu().numpy(), want_types), (nw, ng, fl)
    assert c.error_flags() == 0
    c.close()


@pytest.mark.parametrize("mode,fl", [(0, 4096), (0, 0), (1, 0)])
def test_dense_tile_build_declines_to_the_chains(sh, ctx, full_data, mode, fl):
    """Every child on one gift type: a block's 256 columns share that type,
    more than the packed build's type table holds (255), so the dense-tile
    kernel (mode 0, SH_FLAG_DT_TILE and the few-block default) and the 4-wave
    twins kernel decline their fast build and use the type -> column chains;
    the round equals the oracle's all the same."""
    n, B = 256, 6
    rows = ctx.sample_blocks(mode, n, B, 9, 0)
    t0 = np.zeros_like(full_data.types)
    t_host = t0.copy()
    ocol, ocost = oracle.round_blocks(mode, full_data.wish, t_host, rows.cpu().numpy().reshape(B, n),
                                      ng=full_data.ng)
    types = torch.from_numpy(t0).cuda()  # (one type everywhere: legal per block, not a real state)
    col = torch.empty(B * n, dtype=torch.int32, device="cuda")
    cost = torch.empty(B, dtype=torch.int64, device="cuda")
    ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, flags=fl)
    assert np.array_equal(col.cpu().numpy().reshape(B, n), ocol)
    assert np.array_equal(cost.cpu().numpy(), ocost)
    assert np.array_equal(types.cpu().numpy(), t_host)
    assert ctx.error_flags() == 0


@pytest.mark.parametrize("mode,n,B,fl", [(0, 256, 3730, 0), (0, 256, 466, 0), (0, 256, 64, 32), (0, 256, 64, 8),
                                         (0, 256, 64, 256), (0, 256, 64, 512), (1, 256, 78, 0), (0, 2000, 24, 0),
                                         (0, 600, 8, 8192), (2, 256, 6, 0)])
def test_solve_round_bookkeeping(sh, ctx, full_data, mode, n, B, fl):
    """sh_solve_round (every design, its fallback launch too: SH_FLAG_TEST_RANGE):
    the same solve as sh_solve_blocks, the round's undo record equals the
    starting types at its rows (and scattering it back undoes the round), the
    next round's rows equal sh_sample_blocks' for that round, and the publish
    (folded into the fallback launch, or its own kernel) puts the delta sums
    into the mailbox behind the sequence number and zeroes the delta."""
    _, _, _, nb = ctx.geometry(mode, n)
    rows = ctx.sample_blocks(mode, n, B, 77, 3)
    seq = (1 << 40) + B * 16 + fl % 16 + 4096 * n  # (unique per case)
    mail = ctx.mailbox
    outs = []
    for fused in (False, True):
        types = ctx.upload_types(full_data.types)
        col = torch.empty(B * n, dtype=torch.int32, device="cuda")
        cost = torch.empty(B, dtype=torch.int64, device="cuda")
        delta = torch.zeros(2, dtype=torch.int64, device="cuda")
        if fused:
            undo = torch.full((B * n,), -7, dtype=torch.int16, device="cuda")
            nxt = torch.full((nb * n,), -1, dtype=torch.int32, device="cuda")
            ctx.solve_round(mode, rows, n, types, undo=undo, next_round=(77, 4, nb, nxt), col=col, cost=cost,
                            delta=delta, publish=(1, seq), flags=fl)
            torch.cuda.synchronize()
            assert mail[4] == seq
            assert delta.cpu().tolist() == [0, 0]
            delta = torch.tensor([mail[5], mail[6]], dtype=torch.int64)
        else:
            ctx.solve_blocks(mode, rows, n, types, col=col, cost=cost, delta=delta, flags=fl)
        assert ctx.error_flags() == 0
        outs.append([x.cpu().numpy() for x in (col, cost, delta, types)])
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
    r = rows.cpu().numpy()
    assert np.array_equal(undo.cpu().numpy(), full_data.types[r])
    assert np.array_equal(nxt.cpu().numpy(), ctx.sample_blocks(mode, n, nb, 77, 4).cpu().numpy())
    types = torch.from_numpy(outs[1][3]).cuda()
    ctx.unpack_types(types, rows, undo, mode)
    assert np.array_equal(types.cpu().numpy(), full_data.types)


def test_publish_delta_mailbox(sh, ctx):
    """sh_publish_delta: the delta sums reach the host mailbox behind their
    sequence number (values first, seq last) and the device delta is zeroed
    for its next round; both slots, sequence numbers that repeat a slot's
    previous value are never mistaken for new ones (the engine's are per
    context and increasing)."""
    mail = ctx.mailbox
    d = torch.tensor([123456789012, -987654321], dtype=torch.int64, device="cuda")
    for slot, seq in ((0, 1001), (1, 1002), (0, 1003)):
        d[0] += slot
        want = d.cpu().tolist()
        ctx.publish_delta(d, slot, seq)
        torch.cuda.synchronize()
        assert mail[4 * slot] == seq
        assert [mail[4 * slot + 1], mail[4 * slot + 2]] == want
        assert d.cpu().tolist() == [0, 0]
        d.copy_(torch.tensor(want, dtype=torch.int64))

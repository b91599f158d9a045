"""FusedTrainerBase.autotune() decision logic on the CPU (one process, fake engine / transports):
peer-transport candidates are validated against the RCCL reference before they are timed, a
candidate that times out or computes different sums is marked inf instead of raising, a
failing standalone peer kernel drops every peer candidate, and the training state is put back
after the scratch steps.  The GPU counterpart with real kernels (one rank withholding its
co-scheduled flags) is tests/test_gpu_peer.py::test_autotune_drops_failing_coscheduled_exchange."""
import types

import pytest
import torch

from mxddp.fused import FusedTrainerBase

N = 64


class _Peer:
    def __init__(self, fail=()):
        self.fail = set(fail)   # strategies whose exchange "times out"
        self.err = 0
        self.timeouts = []
        self.resyncs = 0

    def error(self):
        return self.err

    def reset_state(self):
        self.err = 0
        self.resyncs += 1

    def set_timeout_ms(self, ms):
        self.timeouts.append(ms)


class _Eng:
    """Stands in for MnistEngine: a step adds -lr * g to the params, where g is the 'all-reduced'
    gradient; a broken strategy sets the peer's error word and applies garbage."""

    def __init__(self, tr, wrong=()):
        self.tr, self.wrong = tr, set(wrong)
        self.reducer_active = True
        self.peer = None
        self.strat = "ovl"
        self.counter_ptr = tr.workspace.data_ptr()
        self.captured = False
        self.graph_mode = 0
        self.launches = []

    def uncapture(self):
        self.captured = False

    def capture(self, mode, spg):
        self.captured = True

    def set_peer(self, p):
        self.peer = p

    def set_comm(self, c):
        pass

    def set_bucket_padding(self, n, mult):
        pass

    def set_merged(self, on):
        if on:
            self.strat = "one"

    def set_overlap(self, on):
        if on:
            self.strat = "ovl"
        elif self.strat == "ovl":
            self.strat = "inl"

    def set_coscheduled(self, on):
        if on:
            self.strat = "co"
        return on

    def repack(self):
        pass

    def sync(self):
        pass

    def replay(self, n):
        tr = self.tr
        for _ in range(n):
            self.launches.append(("peer" if self.peer else "rccl", self.strat))
            g = torch.linspace(-1, 1, N)
            if self.peer is not None and self.strat in self.peer.fail:
                self.peer.err = 2
                g = torch.zeros(N)
            elif self.peer is not None and self.strat in self.wrong:
                g = g * 1.5
            tr.mom.mul_(0.9).add_(g)
            tr.params.sub_(0.1 * tr.mom)


class _Trainer(FusedTrainerBase):
    LAYOUT = [("w", (N,))]

    def _candidate_strategies(self, transport):
        return ["ovl", "inl", "one"] + (["co"] if transport == "peer" else [])

    def _set_buckets(self, strat):
        self.eng.strat = strat
        self.bucket_strategy = strat

    def _opt_tensors(self):
        return {"mom": self.mom}


def _make(peer_fail=(), wrong=(), with_peer=True):
    tr = _Trainer.__new__(_Trainer)
    tr.device = torch.device("cpu")
    tr.params = torch.randn(N)
    tr.mom = torch.zeros(N)
    tr.metrics = torch.zeros(4)
    tr.workspace = torch.zeros(16)
    tr.comm = types.SimpleNamespace(world_size=2, variant="default", check_async_error=lambda: None)
    tr.eng = _Eng(tr, wrong)
    tr.stream = None
    tr.steps = tr.steps_at_reset = 0
    tr.use_graph, tr._external, tr._capture_done, tr.steps_per_graph = True, False, False, None
    tr.transport, tr.world_size = "auto", 2
    tr.rccl_variants = [("default", tr.comm)]
    tr.eng_comm = tr.comm
    tr._grad_slack = 0
    tr.peer = _Peer(peer_fail) if with_peer else None
    tr._peer_resync = lambda: tr.peer.reset_state() if tr.peer is not None else None
    return tr


def _pc_stub(monkeypatch):
    from mxddp.parallel import comm as pc

    monkeypatch.setattr(pc, "barrier", lambda: None)
    monkeypatch.setattr(pc, "all_reduce_max", lambda v: v)


def test_failing_coscheduled_strategy_is_dropped_not_raised(monkeypatch):
    _pc_stub(monkeypatch)
    tr = _make(peer_fail={"co"})
    res = tr.autotune(trial_steps=3)
    co = [v for k, v in res.items() if k[0] == "peer" and k[2] == "co"]
    assert co and all(v == float("inf") for v in co)
    assert tr.tuned["peer_validated"]["co"] is False
    assert tr.tuned["buckets"] != "co"
    # the other peer strategies still ran and were timed
    assert any(k[0] == "peer" and v < float("inf") for k, v in res.items())
    assert tr.peer.timeouts[0] == 2000.0 and tr.peer.timeouts[-1] == 30000.0  # short while tuning
    assert tr.peer.err == 0


def test_wrong_sums_fail_validation(monkeypatch):
    _pc_stub(monkeypatch)
    tr = _make(wrong={"co"})
    res = tr.autotune(trial_steps=3)
    assert all(v == float("inf") for k, v in res.items() if k[2] == "co")
    assert tr.tuned["peer_validated"] == {"ovl": True, "inl": True, "one": True, "co": False}


def test_broken_standalone_peer_drops_every_peer_candidate(monkeypatch):
    _pc_stub(monkeypatch)
    tr = _make(peer_fail={"ovl", "inl", "one", "co"})
    res = tr.autotune(trial_steps=3)
    assert all(v == float("inf") for k, v in res.items() if k[0] == "peer")
    assert tr.tuned["transport"].startswith("rccl")
    # only the first standalone strategy was ever run over the peer transport
    assert {s for t, s in tr.eng.launches if t == "peer"} == {"ovl"}


def test_validation_steps_do_not_train(monkeypatch):
    """The validation and reference steps are scratch: with restore=True the trainer ends exactly
    where it started."""
    _pc_stub(monkeypatch)
    tr = _make()
    p0 = tr.params.clone()
    tr.autotune(trial_steps=2, restore=True)
    assert torch.equal(tr.params, p0) and tr.steps == 0
    assert tr.discarded_steps > 0


def test_no_working_candidate_raises(monkeypatch):
    _pc_stub(monkeypatch)
    tr = _make(peer_fail={"ovl", "inl", "one", "co"})
    tr.transport = "peer"  # peer-only job (ranks share a GPU): nothing else to fall back to
    with pytest.raises(RuntimeError, match="no launch strategy"):
        tr.autotune(trial_steps=2)


def test_rccl_variant_that_fails_to_initialise_is_dropped(monkeypatch, capsys):
    """An RCCL communicator variant the library refuses (ncclCommInitRankConfig error) is dropped
    from the candidates on every rank (the verdict is agreed), with the reason logged -- not an
    exception that kills the bench."""
    from mxddp.parallel import comm as pc

    _pc_stub(monkeypatch)
    tr = _make()
    tr.rccl_variants = None
    good = types.SimpleNamespace(world_size=2, variant="Ring:c28")

    def fake_rccl_comm(force=False, variant="default"):
        if variant == "Ring:c7":
            raise RuntimeError("ncclCommInitRankConfig: invalid argument")
        return good

    monkeypatch.setattr(pc, "rccl_variants", lambda: ["default", "Ring:c7", "Ring:c28"])
    monkeypatch.setattr(pc, "rccl_comm", fake_rccl_comm)
    cands = tr._rccl_candidates()
    assert list(cands) == ["default", "Ring:c28"] and cands["Ring:c28"] is good
    assert "RCCL variant 'Ring:c7' dropped" in capsys.readouterr().err


def test_autotune_restores_without_restore_flag(monkeypatch):
    """Trial steps are scratch whatever ``restore`` says: the state after autotune does not depend
    on which candidates ran (restore=False used to keep some candidates' steps)."""
    _pc_stub(monkeypatch)
    tr = _make(wrong={"co"})
    p0 = tr.params.clone()
    tr.autotune(trial_steps=2, restore=False)
    assert torch.equal(tr.params, p0) and tr.steps == 0 and tr.discarded_steps > 0


def test_autotune_wall_time_budget_skips_the_rest(monkeypatch, capsys):
    """Once the (agreed) elapsed time passes the budget, the remaining candidates are skipped on
    every rank and listed; the best of those timed is chosen."""
    _pc_stub(monkeypatch)
    tr = _make()
    res = tr.autotune(trial_steps=2, budget_s=0.0)
    timed = [k for k, v in res.items() if v < float("inf")]
    assert len(timed) == 1 and tr.tuned["skipped"]  # the first candidate always runs
    assert len(res) + len(tr.tuned["skipped"]) > 1
    assert "budget reached" in capsys.readouterr().err
    assert f"{timed[0][0]}/{timed[0][1]}/{timed[0][2]}" == f"{tr.tuned['transport']}/{tr.tuned['graph_mode']}/{tr.tuned['buckets']}"


def test_rejection_names_the_differing_tensors():
    """A rejected peer candidate's message says which parameter tensors (and what fraction of
    each) disagree with the reference steps, so a failure in a log points at a bucket."""
    obj = types.SimpleNamespace(LAYOUT=[("a.weight", (4, 2)), ("a.bias", (4,)), ("b.weight", (2, 2))])
    ref = torch.ones(16 + 16)  # params (16) + optimizer state (16)
    d = ref.clone()
    d[8:10] += 1.0             # half of a.bias
    d[30] = 5.0                # optimizer state
    msg = FusedTrainerBase._where_differs(obj, d, ref)
    assert msg == "differing: a.bias 50%, optimizer state 6%", msg
    assert FusedTrainerBase._where_differs(obj, ref.clone(), ref) == "differing: none"

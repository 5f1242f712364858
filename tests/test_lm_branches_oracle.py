"""CPU: the oracle's Levenberg-Marquardt bookkeeping on the branch-forcing
cases of tests/lm_cases.py, against the committed fixtures
tests/golden/lm_branches.{json,npz} (made by tests/golden/make_lm_branches.py,
which cross-checked every trajectory against an independent dense numpy
restatement of Ceres-1.12's trust-region loop: same accept / reject / invalid
sequence and termination).

Parity is UNPINNED against Ceres itself (absent): these tests
pin the oracle to the restatement it was checked against and to itself.
"""
import json
import os

import numpy as np
import pytest

import lm_cases as L
from oracle import ffi as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIX = json.load(open(os.path.join(G, "lm_branches.json")))
ARR = np.load(os.path.join(G, "lm_branches.npz"))
SEQ = {"CONVERGENCE": 0, "NO_CONVERGENCE": 1, "FAILURE": 2}


def seq_of(trace):
    return "".join("I" if not it["step_is_valid"] else ("A" if it["step_is_successful"] else "R") for it in trace[1:])


def test_every_branch_is_covered():
    seqs = {n: seq_of(c["trace"]) for n, c in FIX.items()}
    terms = {c["summary"]["termination_type"] for c in FIX.values()}
    assert terms == {0, 1, 2}                                    # CONVERGENCE, NO_CONVERGENCE, FAILURE
    assert any("R" in s for s in seqs.values())                 # rejected steps
    assert any("RRR" in s for s in seqs.values())               # consecutive rejections (decrease factor 8)
    assert any("I" in s for s in seqs.values())                 # invalid steps (LLT failure)
    assert seqs["gradient_initial"] == ""                        # gradient test at iteration 0
    assert FIX["no_convergence"]["summary"]["num_iterations"] == FIX["no_convergence"]["options"]["max_num_iterations"]
    assert FIX["llt_invalid_3"]["summary"]["num_invalid_steps"] == 3
    # the max_trust_region_radius clamp is reached exactly
    assert any(it["trust_region_radius"] == 1e16 for it in FIX["gauge_1e16"]["trace"])


@pytest.mark.parametrize("name", sorted(FIX))
def test_oracle_reproduces_fixture(name):
    c = FIX[name]
    build, _, mode = L.cases()[name]
    s = build()
    assert s.n_obs == c["n_obs"]
    r, t, X = s.copy_params()
    sm, tr = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, mode=mode, options=O.default_options(**c["options"]))
    assert sm["termination_type"] == c["summary"]["termination_type"]
    assert seq_of(tr) == seq_of(c["trace"])
    for a, b in zip(tr, c["trace"]):
        assert abs(a["cost"] - b["cost"]) <= 1e-12 * b["cost"]
        assert abs(a["trust_region_radius"] - b["trust_region_radius"]) <= 1e-12 * b["trust_region_radius"]
    for k, v in (("rot", r), ("t", t), ("X", X)):
        ref = ARR[f"{name}__{k}"]
        assert np.max(np.abs(v - ref) / np.maximum(np.abs(ref), 1e-3)) < 1e-10
    # the independent numpy restatement agreed when the fixture was made
    k = c["decisive_prefix"]
    assert c["numpy_sequence"][:k] == seq_of(c["trace"])[:k]
    if not name.startswith("gauge"):
        assert c["numpy_sequence"] == seq_of(c["trace"])
        assert SEQ[c["numpy_termination"]] == c["summary"]["termination_type"]


def test_radius_bookkeeping_of_consecutive_rejections():
    """radius /= decrease_factor, decrease_factor *= 2 on every rejection
    (reset to 2 on acceptance): three rejections in a row divide the radius
    by 2, 4 and 8 (LevenbergMarquardtStrategy::StepRejected)."""
    tr = FIX["reject_a"]["trace"]
    s = seq_of(tr)
    i = s.index("RRR") + 1
    r = [it["trust_region_radius"] for it in tr]
    assert r[i] == pytest.approx(r[i - 1] / 2, rel=1e-15)
    assert r[i + 1] == pytest.approx(r[i] / 4, rel=1e-15)
    assert r[i + 2] == pytest.approx(r[i + 1] / 8, rel=1e-15)


def test_invalid_steps_halve_the_radius_and_keep_the_parameters():
    c = FIX["llt_invalid"]
    r = [it["trust_region_radius"] for it in c["trace"]]
    assert r[:5] == [1e4, 5e3, 1.25e3, 1.5625e2, 9.765625]
    s = L.on_axis_scene()
    for k, v in (("rot", s.rot), ("t", s.t), ("X", s.X)):
        assert np.array_equal(ARR[f"llt_invalid__{k}"], v)


@pytest.mark.parametrize("bad", [dict(min_lm_diagonal=-1.0), dict(max_lm_diagonal=1e-9),
                                 dict(min_trust_region_radius=2e4), dict(initial_trust_region_radius=0.0),
                                 dict(function_tolerance=-1.0), dict(max_num_iterations=-1)])
def test_oracle_refuses_invalid_options(bad):
    s = L.reject_scene("reject_a")
    r, t, X = s.copy_params()
    with pytest.raises(RuntimeError, match="-22"):
        O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, options=O.default_options(**bad))


@pytest.mark.parametrize("name", sorted(n for n in FIX if not n.startswith("gauge")))
def test_oracle_summation_order_variant_takes_the_same_branches(name):
    """oracle order=1 (the reduced matrix's diagonal blocks summed in the
    device solver's association: the same arithmetic in another valid order)
    takes every branch scene's decisions as the Ceres order does; the gauge
    scenes are where it does not (tests/test_gpu_lm_branches.py,
    profiles/r04_gauge_order_probe.txt)."""
    c = FIX[name]
    build, _, mode = L.cases()[name]
    s = build()
    out = []
    for order in (0, 1):
        r, t, X = s.copy_params()
        sm, tr = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, mode=mode,
                         options=O.default_options(**c["options"]), order=order)
        out.append((sm, tr))
    (s0, t0), (s1, t1) = out
    seq = lambda tr: [(it["step_is_valid"], it["step_is_successful"]) for it in tr]
    assert seq(t0) == seq(t1)
    assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-8 * s0["final_cost"]

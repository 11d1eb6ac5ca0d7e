"""NARX / ML backends (CPU): ANN translation, lifted stage NLP, oracle solve.

The reference pins the ANN translation only against keras (to 5 decimals,
`tests/test_serialized_ann.py:80-90`, keras absent here), and the NARX
transcription only by running the three-zone example; the checks below pin
(a) the symbolic ANN against its numpy forward pass, (b) the product's
reference-layout NLP against the oracle restatement (`tests/test_transcription.py`
runs ``room_nn``), and (c) the kernel's lifted stage NLP against the
reference-layout NLP at random points, plus an oracle IPM solve of C5.
"""

import json

import numpy as np
import pytest

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.data_structures import ml_model_datatypes as mlt
from agentlib_mpc_amd.models import examples as ex
from agentlib_mpc_amd.models.casadi_predictor import CasadiANN
from agentlib_mpc_amd.models.serialized_ml_model import SerializedANN, SerializedMLModel
from oracle import ipm
from tests import configs


def test_column_order_and_lag_names():
    """`ml_model_datatypes.py:118-138` on the three-zone T_air network."""
    ann = ex.room_cca_anns()[0]
    cols = mlt.column_order(ann.input, ann.output)
    assert cols == ["T_CCA_0", "T_ahu", "mDot_ahu", "d", "d_1", "T_amb", "Q_rad", "Q_rad_1", "T_air"]
    assert mlt.name_with_lag("x", 0) == "x" and mlt.name_with_lag("x", 2) == "x_2"
    with pytest.raises(ValueError):
        mlt.OutputFeature(name="y", output_type="difference", recursive=False)


def test_symbolic_ann_matches_numpy_and_json_round_trip():
    ann = ex.room_cca_anns()[1]
    again = SerializedMLModel.load_serialized_model(json.loads(ann.model_dump_json()))
    assert isinstance(again, SerializedANN)
    net, net2 = CasadiANN(ann), CasadiANN(again)
    rng = np.random.default_rng(3)
    xs = np.array([296.0, 295.0, 294.0, 293.0, 120.0, 0.1, 0.08, 295.5]) + rng.normal(size=(5, 8))
    syms = [sx.sym(f"u{i}") for i in range(8)]
    out = net.predict(syms)
    for x in xs:
        got = float(sx.evaluate(out, dict(zip(syms, x)))[0])
        # normalisation is folded into the first layer: agreement to rounding
        np.testing.assert_allclose(got, net.predict_numpy(x)[0, 0], rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(net2.predict_numpy(x), net.predict_numpy(x), rtol=0, atol=0)


def test_network_node_derivatives_match_expanded_graph():
    """The opaque network node (value, gradient, Hessian via symbolic AD rules) ==
    the layer-by-layer expanded graph differentiated by the generic AD."""
    ann = ex.room_cca_anns()[0]
    net = CasadiANN(ann)
    xs = [sx.sym(f"x{i}") for i in range(net.n_in)]
    opaque = net.predict(xs)[0]
    assert opaque.op.startswith("annv")
    expanded = xs
    for spec in net.layers:
        expanded = CasadiANN._layer_sym(spec, expanded)
    expanded = expanded[0]
    sel = [0, 1, 8]  # differentiate w.r.t. a few inputs
    outs = []
    for e in (opaque, expanded):
        g = [sx.diff(e, xs[i]) for i in sel]
        h = [sx.diff(gi, xs[j]) for gi in g for j in sel]
        outs.append([e] + g + h)
    x = np.array([295.5, 296.0, 0.03, 120.0, 110.0, 300.0, 90.0, 80.0, 296.2])
    vals = dict(zip(xs, x))
    a = np.array(sx.evaluate(outs[0], vals), float)
    b = np.array(sx.evaluate(outs[1], vals), float)
    np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name,kw", [("room_nn", {}), ("room_nn", {"N": 23}), ("one_room_du", {})])
def test_lifted_stage_nlp_reproduces_reference_nlp(name, kw):
    """Kernel stage form == reference NLP: NARX super-stages (N=24), NARX copy-lifting
    (N=23, lag-window copies + shift constraints) and carried previous controls of
    change penalties (copy of u_{k-1} in the stage state, X_0[u] = u_prev)."""
    case = configs.CASES[name](**kw)
    prob = case.backend.problem
    nlp, lift, st = prob.nlp, prob.nlp.lift, prob.nlp.stage
    (p, lbw, ubw, w0), _ = configs.product_nlp_inputs(case)
    rng = np.random.default_rng(5)
    w = w0 + rng.normal(scale=0.5, size=w0.shape) * (lbw < ubw)
    vals = {s: v for s, v in zip(nlp.w_syms, w)}
    vals.update({s: v for s, v in zip(nlp.p_syms, p)})
    ref = np.array(sx.evaluate([nlp.f_expr] + nlp.g_exprs, vals), float)
    kp, kl, ku, kw = prob.to_kernel(p, lbw, ubw, w)
    assert len(kw) == nlp.kernel_nw and len(kp) == nlp.kernel_np
    assert np.all(np.isinf(kl[lift.w_dup])) and np.all(np.isinf(ku[lift.w_dup]))
    npb = nlp.nv + nlp.nx
    ftot, g = 0.0, []
    for k in range(nlp.N):
        loc = kw[k * npb: k * npb + len(st.local)]
        sv = dict(zip(st.local, loc))
        sv.update(zip(st.PS, kp[nlp.npg + k * nlp.nps: nlp.npg + (k + 1) * nlp.nps]))
        sv.update(zip(st.PG, kp[:nlp.npg]))
        sv[st.TK] = k * nlp.ts
        out = sx.evaluate([st.cost] + st.g, sv)
        ftot += float(out[0])
        g += [float(v) for v in out[1:]]
    g = np.array(g)
    np.testing.assert_allclose(ftot, ref[0], rtol=1e-13)
    np.testing.assert_allclose(g[lift.g_of_ref], ref[1:], rtol=1e-12, atol=1e-9)
    shift = np.setdiff1d(np.arange(len(g)), lift.g_of_ref)
    np.testing.assert_array_equal(g[shift], 0.0)  # copies are consistent at mapped points
    # the reference solution is recovered from the kernel vector
    np.testing.assert_array_equal(prob.from_kernel(kw, lbw), np.where(lift.w_primary >= 0, w, lbw))


def test_lags_per_variable_and_backend_keys():
    case = configs.room_nn()
    be = case.backend
    # `casadi_ml.py:387-397`: every lagged feature in the var_ref, (lag - 1) * ts
    assert be.get_lags_per_variable() == {
        "T_CCA_0": 0.0, "T_ahu": 0.0, "mDot_ahu": 0.0, "d": 1800.0, "T_amb": 0.0, "Q_rad": 1800.0,
        "T_air": 0.0, "T_v": 3600.0, "mDot": 1800.0}
    assert len(be.coupling_grid) == 24
    from agentlib_mpc_amd.optimization_backends import backend_types
    for key in ("casadi_ml", "casadi_nn", "casadi_admm_ml", "casadi_admm_nn"):
        assert key in backend_types


def test_ml_model_config_errors():
    ann_air, ann_cca = ex.room_cca_anns()
    with pytest.raises(ValueError, match="same output"):
        ex.RoomCCA(ml_model_sources=[ann_air, ann_air], dt=1800)
    bad = ann_air.model_copy(deep=True)
    bad.input = dict(bad.input)
    bad.input["nonexistent"] = mlt.Feature(name="nonexistent")
    with pytest.raises(ValueError, match="do not appear"):
        ex.RoomCCA(ml_model_sources=[bad, ann_cca], dt=1800)


@pytest.mark.slow
def test_oracle_solves_room_nn():
    case = configs.room_nn()
    p, lbw, ubw, w0 = case.oracle_inputs
    fn = case.oracle.functions(p)
    res = ipm.solve(fn, w0, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p), ipm.IPMOptions(tol=1e-10, acceptable_iter=0))
    assert res.success, res.status
    r = fn.grad_f(res.x) + fn.jac_g(res.x).T @ res.lam_g + res.lam_x
    free = lbw < ubw  # fixed past values are parameters (IPOPT make_parameter)
    assert np.max(np.abs(r[free])) < 1e-9 * max(1.0, np.max(np.abs(fn.grad_f(res.x))))

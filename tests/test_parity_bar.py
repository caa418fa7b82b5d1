"""The history parity bar itself (tests/parity.py), on synthetic histories: the strict 1e-12
bar, the named drift fallback with its per-row running envelope, and the margin log."""

import json

import numpy as np
import pytest

from tests import parity


@pytest.fixture(autouse=True)
def log_path(tmp_path, monkeypatch):
    p = tmp_path / "margins.jsonl"
    monkeypatch.setenv("MIGMRES_PARITY_LOG", str(p))
    return p


def _recs(p):
    return [json.loads(line) for line in open(p)]


def test_strict_bar_passes_and_logs(log_path):
    ref = np.linspace(1.0, 1e-9, 12).reshape(6, 2)
    parity.hist_close(ref + 5e-13, ref)
    (r,) = _recs(log_path)
    assert r["strict_ok"] and not r["fallback_used"] and r["max_abs_diff"] == pytest.approx(5e-13, rel=1e-3)


def test_unnamed_case_cannot_use_drift(log_path):
    ref = np.linspace(1.0, 1e-9, 12).reshape(6, 2)
    with pytest.raises(AssertionError, match="not named restart-sensitive"):
        parity.hist_close(ref + 3e-12, ref, ref + 1e-12)
    assert _recs(log_path)[0]["passed"] is False


def test_drift_envelope_is_per_row(log_path):
    ref = np.linspace(1.0, 1e-9, 8).reshape(4, 2)
    ref2 = ref.copy()
    ref2[2, 0] += 1e-12          # the oracle's own drift appears at row 2
    ok = ref.copy()
    ok[3, 1] += 8e-12            # after it: within 1e-12 + 10 x envelope
    parity.hist_close(ok, ref, ref2, drift_ok=True)
    bad = ref.copy()
    bad[1, 0] += 8e-12           # before the drift appears: the envelope is still 0
    with pytest.raises(AssertionError, match="row 1"):
        parity.hist_close(bad, ref, ref2, drift_ok=True)
    recs = _recs(log_path)
    assert recs[0]["fallback_used"] and recs[0]["passed"] and recs[0]["worst_row"] == 3
    assert recs[1]["passed"] is False


def test_true_residual_bar(log_path):
    parity.true_residuals_close(np.array([1e-9, 2e-9]), np.array([1e-9 + 1e-12, 2e-9]), 0.0)
    with pytest.raises(AssertionError):
        parity.true_residuals_close(np.array([1e-9]), np.array([1.1e-9]), 0.0)

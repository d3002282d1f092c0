"""Data pipeline: EDF round trip, XML parsing (stop at first stage), windowing/labels vs a naive
statement of the reference rule, standardisation, SMOTE/RUS properties, cohort descriptives."""
import numpy as np
import pandas as pd
import pytest

from uncertaintyquantification_sleepapnea_1dcnn_amd.data import annotations, balance, cohort, edf, preprocess, prepare


def test_edf_roundtrip(tmp_path):
    rs = np.random.RandomState(0)
    sig = {"SaO2": 90 + rs.rand(600) * 10, "THOR RES": rs.randn(6000)}
    p = edf.write_edf(str(tmp_path / "a.edf"), sig, {"SaO2": 1.0, "THOR RES": 10.0},
                      phys_ranges={"SaO2": (0, 100), "THOR RES": (-5, 5)})
    got, rates = edf.read_edf(p)
    assert rates == {"SaO2": 1.0, "THOR RES": 10.0}
    np.testing.assert_allclose(got["SaO2"], sig["SaO2"], atol=100 / 65535)
    np.testing.assert_allclose(got["THOR RES"], sig["THOR RES"], atol=10 / 65535)


def test_xml_stops_at_first_stage(tmp_path):
    ev = [{"event_concept": "Recording Start Time", "start": 0, "duration": 20000.0},
          {"event_concept": "Hypopnea|Hypopnea", "start": 100.0, "duration": 15.0}]
    p = annotations.write_xml_annotations(str(tmp_path / "a.xml"), ev)
    got = annotations.parse_xml_annotations(p)
    assert [e["event_concept"] for e in got] == ["Recording Start Time", "Hypopnea|Hypopnea"]
    assert annotations.calculate_sleep_time(got) is True
    with pytest.raises(KeyError):  # the reference's key-name bug, reproducible on request (Q7)
        annotations.calculate_sleep_time(got, reference_keys=True)


def test_windowing_matches_naive_rule():
    rs = np.random.RandomState(1)
    n = 60 * 20 + 37
    df = pd.DataFrame({c: rs.randn(n) for c in ["SaO2", "PR", "THOR RES", "ABDO RES"]})
    ev = pd.DataFrame([{"event_concept": "Obstructive apnea|Obstructive Apnea", "start": 55.0, "duration": 12.0},
                       {"event_concept": "Hypopnea|Hypopnea", "start": 170.0, "duration": 9.0},
                       {"event_concept": "Central apnea|Central Apnea", "start": 300.0, "duration": 30.0},
                       {"event_concept": "Hypopnea|Hypopnea", "start": 415.0, "duration": 30.0}])
    out = preprocess.segment_and_label_edf_data(df, ev, "p1")
    assert len(out) == 20 and list(out.columns[:5]) == ["SaO2_t0", "PR_t0", "THOR RES_t0", "ABDO RES_t0", "SaO2_t1"]
    for i in range(20):
        s, e = 60 * i, 60 * i + 60
        lab = 0
        for _, r in ev.iterrows():
            if r["event_concept"] in annotations.APNEA_EVENTS:
                if min(e, r["start"] + r["duration"]) - max(s, r["start"]) >= 10:
                    lab = 1
                    break
        assert out["Apnea/Hypopnea"].iloc[i] == lab
        np.testing.assert_allclose(out.iloc[i, :240].to_numpy(float), df.iloc[s:e].to_numpy().reshape(-1))


def test_artifact_interpolation():
    s = {"SaO2": np.array([95.0, 50.0, 97.0, 99.0]), "PR": np.array([60.0, 70.0, 300.0, 80.0])}
    out = preprocess.remove_artifacts(s)
    np.testing.assert_allclose(out["SaO2"], [95, 96, 97, 99])
    np.testing.assert_allclose(out["PR"], [60, 70, 75, 80])


def test_standardize_per_window():
    x = np.random.RandomState(2).randn(10, 60, 4) * 3 + 7
    z = prepare.standardize_per_window(x, device="cpu")
    np.testing.assert_allclose(z.mean(1), 0, atol=1e-9)
    np.testing.assert_allclose(z.std(1), 1, atol=1e-6)


def test_smote_and_rus():
    rs = np.random.RandomState(0)
    X = rs.randn(300, 12)
    y = (rs.rand(300) < 0.2).astype(int)
    Xs, ys = balance.SMOTE(random_state=2025, knn_device="sklearn").fit_resample(X, y)
    assert np.bincount(ys)[0] == np.bincount(ys)[1]
    np.testing.assert_array_equal(Xs[:300], X)  # originals first, synthetic appended (Q5)
    Xm = X[y == 1]
    nn = balance.knn_indices(Xm, 5, "sklearn")
    for xnew in Xs[300:310]:  # every synthetic point lies on a segment to one of the 5 neighbours
        ok = False
        for i in range(len(Xm)):
            for j in nn[i]:
                d = Xm[j] - Xm[i]
                t = np.dot(xnew - Xm[i], d) / np.dot(d, d)
                if 0 <= t <= 1 and np.allclose(Xm[i] + t * d, xnew, atol=1e-9):
                    ok = True
        assert ok
    Xs2, _ = balance.SMOTE(random_state=2025, knn_device="sklearn").fit_resample(X, y)
    np.testing.assert_array_equal(Xs, Xs2)  # deterministic for a seed
    Xu, yu = balance.RandomUnderSampler(random_state=2025).fit_resample(X, y)
    assert np.bincount(yu)[0] == np.bincount(yu)[1] == np.bincount(y)[1]
    assert list(yu[: np.bincount(yu)[0]]) == [0] * np.bincount(yu)[0]


def test_cohort_descriptives(tmp_path):
    p = tmp_path / "shhs2.csv"
    pd.DataFrame({"ahi_a0h3a": [2.0, 7.0, 20.0, 40.0, np.nan], "age_s2": [60, 70, 65, 80, 50],
                  "gender": [1, 2, 1, 2, 1], "race": [1, 2, 3, 1, 1], "quoxim": [5, 4, 5, 3, 1]}).to_csv(p, index=False)
    r = cohort.analyze_cohort(str(p), verbose=False)
    assert r["n_cohort"] == 4
    assert [r["ahi_categories"]["counts"][k] for k in cohort.AHI_CATEGORIES] == [1, 1, 1, 1]
    q = cohort.analyze_signal_quality(str(p), verbose=False)
    assert q["quoxim"]["counts"] == {3: 1, 4: 1, 5: 2}


def test_pr_fallback_gates_resample_reshape(tmp_path):
    rs = np.random.RandomState(3)
    sig = {"SaO2": 90 + rs.rand(300) * 5, "H.R.": 60 + rs.rand(300) * 20, "THOR RES": rs.randn(3000)}
    p = edf.write_edf(str(tmp_path / "b.edf"), sig, {"SaO2": 1.0, "H.R.": 1.0, "THOR RES": 10.0},
                      phys_ranges={"SaO2": (0, 100), "H.R.": (0, 250), "THOR RES": (-5, 5)})
    s, r = preprocess.get_edf_channels(p, ["SaO2", "PR", "THOR RES"])
    assert set(s) == {"SaO2", "PR", "THOR RES"} and r["PR"] == 1.0  # PR read from H.R.
    np.testing.assert_allclose(s["PR"], sig["H.R."], atol=250 / 65535)
    assert preprocess.check_artifacts_and_missing_values({"a": np.r_[np.ones(95), np.full(5, np.nan)]})
    assert not preprocess.check_artifacts_and_missing_values({"a": np.r_[np.ones(85), np.full(15, np.nan)]})
    out = preprocess.resample_signals({"THOR RES": s["THOR RES"]}, {"THOR RES": 10.0}, 1)
    assert out["THOR RES"].shape == (300,)
    flat = np.arange(2 * 240, dtype=np.float64).reshape(2, 240)  # t-major: SaO2_t0, PR_t0, THOR_t0, ABDO_t0, ...
    x3 = prepare.reshape_flat_to_3d(flat, 60, 4)
    assert x3.shape == (2, 60, 4) and x3[0, 1, 0] == 4 and x3[1, 0, 3] == 243


def test_knn_routes_agree_and_hip_range():
    """The distance-GEMM route (the fallback outside the HIP kernel's k <= 16 / D <= 320 range) agrees
    with the exact search, including for k > 16."""
    assert balance.hip_knn_supported(240, 5) and not balance.hip_knn_supported(240, 17)
    assert not balance.hip_knn_supported(321, 5)
    rs = np.random.RandomState(4)
    X = rs.randn(150, 9)
    for k in (5, 20):
        np.testing.assert_array_equal(balance.knn_indices(X, k, "cpu"), balance.knn_indices(X, k, "sklearn"))

"""Trajectory data format: utils/data_utils.py get_data and
scripts/generate.py post_processed_generated_trajectories.

Pinning: the oracle (oracle/data_ref.py) runs the reference's own lines with the
reference's own dependency (sklearn MinMaxScaler / LabelEncoder, numpy permutation), so
it is the reference's arithmetic; the device scaler, layout transposes and split must equal
it bit for bit (integer/byte-exact bar: float64 sklearn arithmetic, float32 casts).  The
Traffic reader itself (traffic package) is absent: flight grouping is parity unpinned."""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import data_ref

FEATURES = ["latitude", "longitude", "altitude", "timedelta", "groundspeed", "track"]


def _table(n_flights=37, L=50, seed=0):
    rng = np.random.default_rng(seed)
    rows = []
    for i in rng.permutation(n_flights):
        base = rng.normal(size=6) * [10, 10, 3000, 0, 50, 90]
        walk = np.cumsum(rng.normal(size=(L, 6)), 0) * [0.1, 0.1, 100, 1, 2, 5] + base
        walk[:, 3] = np.arange(L) * 4.0
        df = pd.DataFrame(walk, columns=FEATURES)
        df["flight_id"] = f"F{i:04d}"
        df["cluster"] = int(i % 4) * 10 + 3
        rows.append(df)
    return pd.concat(rows, ignore_index=True)


def test_flights_to_arrays_groups_by_flight():
    from timevqvae.utils.data_utils import flights_to_arrays
    df = _table()
    data, labels = flights_to_arrays(df, FEATURES)
    assert data.shape == (37, 50 * 6) and data.dtype == np.float64
    f3 = df[df.flight_id == "F0003"]
    assert np.array_equal(data[3], f3[FEATURES].values.ravel())
    assert labels[3] == 3 * 10 % 40 + 3 or labels[3] == f3.cluster.iloc[0]
    df.loc[df.index[0], "cluster"] = 99
    with pytest.raises(ValueError, match="unique cluster"):
        flights_to_arrays(df, FEATURES)


def test_read_flights_refuses_pickles(tmp_path):
    from timevqvae.utils.data_utils import read_flights
    p = tmp_path / "t.pkl"
    p.write_bytes(b"x")
    with pytest.raises(ValueError, match="pickle"):
        read_flights(str(p))
    q = tmp_path / "t.parquet"
    _table(3, 5).to_parquet(q)
    assert len(read_flights(str(q))) == 15


@pytest.mark.gpu
def test_scaler_equals_sklearn_bitwise(cuda):
    from sklearn.preprocessing import MinMaxScaler
    from timevqvae.utils.data_utils import TrajectoryScaler
    rng = np.random.default_rng(1)
    X = rng.normal(size=(1000, 300)) * rng.uniform(0.1, 1e4, size=300) + rng.normal(size=300) * 1e3
    X[:, 7] = 3.25  # constant column: zero range -> scale 1
    X[5, 11] = np.nan  # skipped by the fit, propagated by the transform
    ref = MinMaxScaler(feature_range=(-1, 1)).fit(X)
    mine = TrajectoryScaler((-1, 1), cuda).fit(X)
    for a in ("data_min_", "data_max_", "data_range_", "scale_", "min_"):
        assert np.array_equal(getattr(mine, a), getattr(ref, a)), a
    want = ref.transform(X).astype(np.float32)
    got = mine.transform(X)
    assert np.array_equal(got, want, equal_nan=True)
    xf = want[:, :].copy()
    assert np.array_equal(mine.inverse_transform(xf), ref.inverse_transform(xf.copy()),
                          equal_nan=True)


@pytest.mark.gpu
def test_get_data_and_postprocess_match_reference(cuda):
    from timevqvae.utils.data_utils import (flights_to_arrays, get_data_from_arrays,
                                            post_processed_generated_trajectories)
    data, labels = flights_to_arrays(_table(), FEATURES)
    train, test, scaler = get_data_from_arrays(data, labels, FEATURES, batch_size=8,
                                               device=cuda, num_workers=0)
    ref_scaler, Xtr, Xte, Ytr, Yte = data_ref.get_data_arrays(data, labels, FEATURES)
    assert torch.equal(train.dataset.X, Xtr) and torch.equal(test.dataset.X, Xte)
    assert torch.equal(train.dataset.Y, Ytr) and torch.equal(test.dataset.Y, Yte)
    assert Xtr.shape[1:] == (6, 50)
    x_gen = Xte + 0.01 * torch.randn_like(Xte)
    x_gen[0, 2] = -5.0  # altitude below the data range -> clipped at 0 after unscaling
    want = data_ref.unscale(x_gen, ref_scaler).reshape(len(x_gen), -1, 6)
    df = post_processed_generated_trajectories(x_gen, Yte, scaler, FEATURES)
    got = np.stack([df[f].values for f in FEATURES], -1).reshape(len(x_gen), -1, 6)
    want[:, :, 2] = np.maximum(want[:, :, 2], 0)
    assert np.array_equal(got, want)
    assert (df.altitude >= 0).all() and df.flight_id.iloc[0] == "TRAJ_0"
    assert (df.cluster.values.reshape(len(x_gen), -1) == Yte.numpy()).all()

"""Trajectory data format (reference utils/data_utils.py:70-138, scripts/generate.py:14-41).

`get_data` reads a flights table, scales it with a MinMax scaler fitted per column to
[-1, 1], lays it out as the model's (N, C, L) and splits it 90/10 with a seed-42
permutation; `post_processed_generated_trajectories` undoes the scaling on generated
samples.  The scaling, the (L, F) <-> (F, L) transposes and the dtype casts run on the
device (csrc/tvq_data.hip), bit-equal to sklearn's MinMaxScaler and numpy's in-place
float32 inverse.

The reference reads the table with `traffic.core.Traffic.from_file` and returns a
`Traffic`.  `traffic` is absent from this image, so tables are read with pandas
(parquet / csv / feather; never pickle) and flights are grouped by `flight_id` in sorted
order (pandas groupby, as Traffic iterates); a `Traffic` is returned when the package is
importable, else the DataFrame.  The flight order of the reference's Traffic iteration
is parity unpinned here."""
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from ..hip._native import call, ptr, stream_ptr, value


def _device(device):
    return torch.device(device) if device is not None else torch.device("cuda")


class TrajectoryScaler:
    """sklearn `MinMaxScaler(feature_range)` semantics with the fit / transform / inverse on
    the device.  Exposes sklearn's fitted attributes (`data_min_`, `data_max_`,
    `data_range_`, `scale_`, `min_`, `n_features_in_`) so the reference's callers
    (`scaler.inverse_transform(x)`, generate.py:17) work unchanged."""

    def __init__(self, feature_range=(-1, 1), device=None):
        self.feature_range = feature_range
        self.device = _device(device)

    # -- sklearn surface ----------------------------------------------------------------
    def fit(self, X):
        X = self._f64(X)
        N, Fc = X.shape
        dev = self.device
        outs = [torch.empty(Fc, dtype=torch.float64, device=dev) for _ in range(4)]
        ws = torch.empty(value("tvq_minmax_fit_workspace", Fc), dtype=torch.float64, device=dev)
        lo, hi = (float(v) for v in self.feature_range)
        call("tvq_minmax_fit", ptr(X), N, Fc, lo, hi, *(ptr(t) for t in outs), ptr(ws),
             stream_ptr())
        self._dmin, self._dmax, self._scale, self._min = outs
        self.data_min_, self.data_max_, self.scale_, self.min_ = (t.cpu().numpy() for t in outs)
        self.data_range_ = self.data_max_ - self.data_min_
        self.n_features_in_ = Fc
        self.n_samples_seen_ = N
        return self

    def transform(self, X):
        """(N, Fc) -> (N, Fc) float32 (sklearn's float64 result, cast as torch.FloatTensor)."""
        X = self._f64(X)
        return self.to_model_layout(X, X.shape[1], 1).reshape(X.shape[0], -1).cpu().numpy()

    def fit_transform(self, X):
        return self.fit(X).transform(X)

    def inverse_transform(self, X):
        """(N, Fc) float32 -> (N, Fc) float32, numpy's in-place `X -= min_; X /= scale_`."""
        x = torch.as_tensor(np.asarray(X, dtype=np.float32)).to(self.device)
        N, Fc = x.shape
        return self.from_model_layout(x.reshape(N, 1, Fc)).cpu().numpy()

    # -- fused device paths ---------------------------------------------------------------
    def to_model_layout(self, X, L, F):
        """(N, L*F) float64 columns [t0 f0, t0 f1, ...] -> scaled (N, F, L) float32 on the
        device: data_utils.py:92-111 (transform, FloatTensor, view (N, L, F), transpose)."""
        X = self._f64(X)
        N, Fc = X.shape
        if Fc != L * F or Fc != self.n_features_in_:
            raise ValueError(f"to_model_layout: {Fc} columns != L*F = {L}*{F} or the fitted "
                             f"{self.n_features_in_}")
        out = torch.empty((N, F, L), dtype=torch.float32, device=self.device)
        call("tvq_minmax_transform", ptr(X), N, L, F, ptr(self._scale), ptr(self._min), ptr(out),
             stream_ptr())
        return out

    def from_model_layout(self, x):
        """(N, F, L) float32 -> unscaled (N, L*F) float32 on the device (generate.py:15-17:
        transpose, reshape, inverse_transform)."""
        x = torch.as_tensor(x).detach().to(self.device, torch.float32).contiguous()
        N, F, L = x.shape
        if L * F != self.n_features_in_:
            raise ValueError(f"from_model_layout: {F}x{L} != the fitted {self.n_features_in_}")
        out = torch.empty((N, L * F), dtype=torch.float32, device=self.device)
        call("tvq_minmax_inverse", ptr(x), N, L, F, ptr(self._scale), ptr(self._min), ptr(out),
             stream_ptr())
        return out

    def _f64(self, X):
        return torch.as_tensor(np.asarray(X) if not torch.is_tensor(X) else X) \
            .to(self.device, torch.float64).contiguous()


class TrajectoryDataset(Dataset):
    """data_utils.py:70-81"""

    def __init__(self, X, Y):
        self.X = X
        self.Y = Y
        self._len = self.X.shape[0]

    def __len__(self):
        return self._len

    def __getitem__(self, idx):
        return self.X[idx], self.Y[idx]


def read_flights(dataset_file: str):
    """A flights table as a DataFrame (parquet, feather or csv; pickles are refused)."""
    import pandas as pd
    ext = os.path.splitext(dataset_file)[1].lower()
    if ext in (".parquet", ".pq"):
        return pd.read_parquet(dataset_file)
    if ext == ".feather":
        return pd.read_feather(dataset_file)
    if ext in (".csv", ".gz"):
        return pd.read_csv(dataset_file)
    raise ValueError(f"read_flights: unsupported table format {ext!r} (pickles are not loaded)")


def flights_to_arrays(df, features):
    """np.stack([f.data[features].values.ravel() for f in traffic]) and the per-flight
    cluster label (data_utils.py:86-101), flights grouped by flight_id, sorted."""
    data, labels = [], []
    for _, f in df.groupby("flight_id"):
        if f["cluster"].nunique() != 1:
            raise ValueError("Each flight should have a unique cluster")
        data.append(f[features].values.ravel())
        labels.append(f["cluster"].iloc[0])
    return np.stack(data).astype(np.float64), np.array(labels)


def get_data_from_arrays(data, labels, features, batch_size: int, train_ratio: float = 0.9,
                         random_seed: int = 42, device=None, num_workers: int = 4):
    """data_utils.py:88-138 from the stacked (N, L*F) array and per-flight labels."""
    from sklearn.preprocessing import LabelEncoder
    F = len(features)
    N, Fc = data.shape
    scaler = TrajectoryScaler(feature_range=(-1, 1), device=device).fit(data)
    X = scaler.to_model_layout(data, Fc // F, F).cpu()  # host tensors, as the reference's
    Y = torch.LongTensor(LabelEncoder().fit_transform(np.asarray(labels).ravel())[:, None])
    np.random.seed(random_seed)
    indices = np.random.permutation(len(X))
    split_idx = int(train_ratio * len(X))
    tr, te = indices[:split_idx], indices[split_idx:]
    train = DataLoader(TrajectoryDataset(X[tr], Y[tr]), batch_size=batch_size, shuffle=True,
                       num_workers=num_workers)
    test = DataLoader(TrajectoryDataset(X[te], Y[te]), batch_size=batch_size, shuffle=False,
                      num_workers=num_workers)
    return train, test, scaler


def get_data(dataset_file: str, features: list, batch_size: int, train_ratio: float = 0.9,
             random_seed: int = 42, device=None):
    """data_utils.py:84-138: (train_loader, test_loader, scaler)."""
    data, labels = flights_to_arrays(read_flights(dataset_file), features)
    return get_data_from_arrays(data, labels, features, batch_size, train_ratio, random_seed,
                                device)


def post_processed_generated_trajectories(x_gen, y_gen, scaler, features):
    """generate.py:14-41: unscale (N, F, L) samples on the device, timedelta of the first
    observation 0, one row per observation with TRAJ_<i> ids and the cluster label,
    altitude clipped at 0, timestamps from timedelta.  Returns a Traffic when the
    `traffic` package is importable, else the DataFrame."""
    import pandas as pd
    x = scaler.from_model_layout(x_gen).cpu().numpy()
    x[:, 3] = 0
    n_samples = x.shape[0]
    x = x.reshape(n_samples, -1, len(features))
    n_obs = x.shape[1]
    df = pd.DataFrame({feature: x[:, :, i].ravel() for i, feature in enumerate(features)})
    ids = np.repeat(np.array([f"TRAJ_{s}" for s in range(n_samples)]), n_obs)
    df = df.assign(flight_id=ids, callsign=ids, icao24=ids)
    labels = torch.as_tensor(y_gen).cpu().numpy()
    df = df.assign(cluster=np.repeat(labels.reshape(n_samples, -1)[:, 0], n_obs))
    if "altitude" in df.columns:
        df.loc[df.altitude < 0, "altitude"] = 0
    if "timedelta" in df.columns:
        base_ts = pd.Timestamp.today(tz="UTC").round(freq="s")
        df = df.assign(timestamp=pd.to_timedelta(df.timedelta, unit="s") + base_ts)
    try:
        from traffic.core import Traffic
    except ImportError:
        return df
    return Traffic(df)

"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's trajectory data format,
using the reference's own dependency (sklearn MinMaxScaler / LabelEncoder) as it does.

* get_data_arrays: utils/data_utils.py:84-124 after the Traffic read (scale, FloatTensor,
  view (N, L, F), transpose, LabelEncoder, seed-42 permutation split).
* unscale: scripts/generate.py:15-18 (transpose, reshape, inverse_transform, timedelta 0).
"""
import numpy as np
import torch
from sklearn.preprocessing import LabelEncoder, MinMaxScaler


def get_data_arrays(data, labels, features, train_ratio=0.9, random_seed=42):
    scaler = MinMaxScaler(feature_range=(-1, 1)).fit(data)
    d = torch.FloatTensor(scaler.transform(data))
    d = torch.transpose(d.view(d.size(0), -1, len(features)), 1, 2)
    y = torch.LongTensor(LabelEncoder().fit_transform(np.asarray(labels).ravel())[:, None])
    np.random.seed(random_seed)
    idx = np.random.permutation(len(d))
    s = int(train_ratio * len(d))
    return scaler, d[idx[:s]], d[idx[s:]], y[idx[:s]], y[idx[s:]]


def unscale(x_gen, scaler):
    x = x_gen.detach().transpose(1, 2).reshape(x_gen.shape[0], -1).cpu().numpy()
    x = scaler.inverse_transform(x)
    x[:, 3] = 0
    return x

"""FID and IS -- the API of the reference timevqvae/evaluation/eval_utils.py.

calculate_fid(z1, z2) (eval_utils.py:56-81): the feature means and sample covariances,
the O(N D^2) part, run on the device in float64 (tvq_fid_moments, csrc/tvq_fid.hip); the
D x D remainder -- sigma1 @ sigma2, its matrix square root (scipy.linalg.sqrtm, real part
when complex) and the trace -- stays on the host in float64 as in the reference.

calculate_inception_score(P_yx, n_split, shuffle, eps) (eval_utils.py:9-53) is host numpy
over an (n, classes) probability table: the exp of the mean KL(p(y|x) || p(y)) per split.
"""
import numpy as np
import torch
from scipy.linalg import sqrtm

from ..hip._native import call, ptr, stream_ptr


def feature_moments(z, device=None):
    """(mu (D,), sigma (D, D)) of the rows of z (N, D): z.mean(0) and
    np.cov(z, rowvar=False), float64 on the device."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    zt = torch.as_tensor(z)
    if zt.dim() != 2 or zt.shape[0] < 2:
        raise ValueError("feature_moments: z must be (N >= 2, D)")
    zt = zt.to(device=dev, dtype=torch.float64).contiguous()
    N, D = zt.shape
    mu = torch.empty(D, device=dev, dtype=torch.float64)
    sigma = torch.empty(D, D, device=dev, dtype=torch.float64)
    call("tvq_fid_moments", ptr(zt), N, D, ptr(mu), ptr(sigma), stream_ptr())
    return mu, sigma


def calculate_fid(z1, z2, device=None):
    """Frechet distance between the Gaussian fits of two feature sets (rows = samples)."""
    mu1, sigma1 = feature_moments(z1, device)
    mu2, sigma2 = feature_moments(z2, device)
    mu1, mu2 = mu1.cpu().numpy(), mu2.cpu().numpy()
    sigma1, sigma2 = sigma1.cpu().numpy(), sigma2.cpu().numpy()
    ssdiff = ((mu1 - mu2) ** 2.0).sum()
    covmean = sqrtm(sigma1.dot(sigma2))
    if np.iscomplexobj(covmean):
        covmean = covmean.real
    return ssdiff + np.trace(sigma1 + sigma2 - 2.0 * covmean)


def calculate_inception_score(P_yx, n_split: int = 10, shuffle: bool = True, eps: float = 1e-16):
    """(mean, std) over n_split splits of exp(E_x KL(p(y|x) || p(y))); shuffles P_yx in
    place with np.random first when `shuffle` (as the reference does)."""
    if shuffle:
        np.random.shuffle(P_yx)
    n_part = int(np.floor(P_yx.shape[0] / n_split))
    scores = []
    for i in range(n_split):
        part = P_yx[i * n_part:(i + 1) * n_part]
        p_y = part.mean(axis=0)[None, :]
        kl = (part * (np.log(part + eps) - np.log(p_y + eps))).sum(axis=1)
        scores.append(np.exp(np.mean(kl)))
    return np.mean(scores), np.std(scores)

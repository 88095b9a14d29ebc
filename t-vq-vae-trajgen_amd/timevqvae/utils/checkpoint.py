"""Checkpoint compatibility with the reference's Lightning checkpoints.

The reference saves `stage{1,2,3}.ckpt` with Lightning (scripts/train.py:115-123) and
loads them with `Stage1.load_from_checkpoint` (maskgit.py:52-59) and
`Stage2.load_from_checkpoint` (generation/sampler.py:76-90).  A Lightning checkpoint is
a dict whose "state_dict" holds the module tree's tensors under the reference's key
names; the modules here keep those names, so loading is `load_state_dict` after
reading the file, plus an adapter for the key-name drift between x-transformers
releases in `transformer_{l,h}.blocks.*` (bidirectional_transformer.py:92-110; the
package is pinned only as `^1.31.6`, pyproject.toml:21).

Files are read with `torch.load(weights_only=True)`: nothing in a checkpoint is
executed.  A checkpoint that holds pickled Python objects is refused with the
loader's own message.
"""
import re

import torch

# x-transformers norm parameter spellings across releases -> the spelling used here
# (RMSNorm `g`, the gamma-only LayerNorm `gamma`)
_NORM_RENAMES = (
    (re.compile(r"(\.attn_layers\.layers\.\d+\.0\.0)\.(gamma|weight)$"), r"\1.g"),
    (re.compile(r"(\.attn_layers\.final_norm)\.(gamma|weight)$"), r"\1.g"),
    (re.compile(r"(\.post_emb_norm)\.(g|weight)$"), r"\1.gamma"),
)
# parameters some releases carry that the restated encoder does not have: accepted only
# when they are the identity (zero bias), as a trained model with them could not be
# reproduced here
_DROP_IF_ZERO = (
    re.compile(r"\.post_emb_norm\.(beta|bias)$"),
    re.compile(r"\.blocks\.project_(in|out)\.bias$"),
)


def read_state_dict(checkpoint_path, map_location="cpu", weights_only=True):
    """The tensors of a Lightning checkpoint ({"state_dict": ...}) or of a bare state_dict."""
    ckpt = torch.load(checkpoint_path, map_location=map_location, weights_only=weights_only)
    if isinstance(ckpt, dict) and "state_dict" in ckpt:
        ckpt = ckpt["state_dict"]
    if not isinstance(ckpt, dict):
        raise ValueError(f"{checkpoint_path}: neither a Lightning checkpoint nor a state_dict")
    return ckpt


def adapt_state_dict(sd, model):
    """Map a reference state_dict onto `model`'s key names.

    Applies the x-transformers norm renames for keys the model does not have verbatim and
    drops identity-valued parameters the restated encoder lacks (raises ValueError for a
    non-zero one).  Keys are otherwise passed through unchanged, so `load_state_dict`'s
    strict check still reports anything missing or unexpected."""
    want = set(model.state_dict().keys())
    out = {}
    for k, v in sd.items():
        if k in want:
            out[k] = v
            continue
        nk = k
        for pat, rep in _NORM_RENAMES:
            nk = pat.sub(rep, nk)
        if nk in want:
            out[nk] = v
            continue
        if any(p.search(k) for p in _DROP_IF_ZERO):
            if torch.count_nonzero(v) != 0:
                raise ValueError(f"checkpoint key {k}: non-zero parameter has no counterpart in "
                                 "the restated x-transformers encoder")
            continue
        out[k] = v
    return out


def save_checkpoint(module, path, **extra):
    """A Lightning-shaped checkpoint ({"state_dict": ..., **extra}) loadable by the
    reference's `load_from_checkpoint` and by this package's."""
    torch.save({"state_dict": module.state_dict(), **extra}, path)

"""TrainedModelSampler, sampling half (reference generation/sampler.py:26-169).

Same constructor and `sample(n_samples, kind, class_index)` contract: Stage2 (with its
frozen Stage1) is loaded from the reference's checkpoints, the FidelityEnhancer from
`stage3.ckpt`'s `fidelity_enhancer.*` entries, and sampling runs MaskGIT iterative
decoding, LF/HF decoding and the FidelityEnhancer on the HIP path.  The evaluation half
(FCN features, FID/IS, PCA/t-SNE plots; do_evaluate=True) is evaluation outside the hot
path and raises here."""
from typing import Union

import torch
import torch.nn as nn

from ..models import FidelityEnhancer
from ..trainers import Stage2
from ..utils.sample_utils import conditional_sample, unconditional_sample
from ..utils.checkpoint import read_state_dict


class TrainedModelSampler(nn.Module):
    def __init__(self, stage1_ckpt_fname, stage2_ckpt_fname, stage3_ckpt_fname, fcn_ckpt_fname,
                 input_length: int, in_channels: int, n_classes: int, batch_size: int,
                 X_train=None, Y_train=None, X_test=None, Y_test=None, device=None,
                 config: dict = None, use_fidelity_enhancer: bool = True,
                 feature_extractor_type: str = "supervised_fcn", rocket_num_kernels: int = 1000,
                 do_evaluate: bool = True):
        super().__init__()
        assert feature_extractor_type in ["supervised_fcn", "rocket"], \
            "unavailable feature extractor type."
        if do_evaluate:
            raise NotImplementedError(
                "TrainedModelSampler(do_evaluate=True): the FCN/FID/IS/PCA evaluation half of "
                "generation/sampler.py is outside the HIP hot path; pass do_evaluate=False "
                "(ROCKET features: timevqvae.evaluation.apply_kernels)")
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.config = config
        self.X_train, self.Y_train, self.X_test, self.Y_test = X_train, Y_train, X_test, Y_test
        self.batch_size = batch_size
        self.feature_extractor_type = feature_extractor_type
        self.stage2 = Stage2.load_from_checkpoint(
            stage2_ckpt_fname, stage1_ckpt_fname=stage1_ckpt_fname, fcn_ckpt_fname=fcn_ckpt_fname,
            input_length=input_length, in_channels=in_channels, n_classes=n_classes,
            X_train=X_train, X_test=X_test, config=config, device=device,
            feature_extractor_type=feature_extractor_type, map_location="cpu")
        self.stage2.eval()
        self.maskgit = self.stage2.maskgit
        self.stage1 = self.stage2.maskgit.stage1
        if use_fidelity_enhancer:
            self.fidelity_enhancer = FidelityEnhancer(input_length=input_length,
                                                      in_channels=in_channels, config=config)
            sd = read_state_dict(stage3_ckpt_fname, map_location="cpu")
            self.fidelity_enhancer.load_state_dict(
                {k.replace("fidelity_enhancer.", ""): v for k, v in sd.items()
                 if k.startswith("fidelity_enhancer.")})
            self.fidelity_enhancer.eval()
        else:
            self.fidelity_enhancer = nn.Identity()
        self.to(self.device)

    @torch.no_grad()
    def sample(self, n_samples: int, kind: str, class_index: Union[int, None] = None):
        """sampler.py:140-169 -> ((x_new_l, x_new_h, x_new), X_new_R), all (b c l) on host."""
        assert kind in ["unconditional", "conditional"]
        if kind == "unconditional":
            x_new_l, x_new_h, x_new = unconditional_sample(self.maskgit, n_samples, self.device,
                                                           batch_size=self.batch_size)
        else:
            x_new_l, x_new_h, x_new = conditional_sample(self.maskgit, n_samples, self.device,
                                                         class_index, self.batch_size)
        out = []
        for start in range(0, x_new.shape[0], self.batch_size):
            mini = x_new[start:start + self.batch_size]
            out.append(self.fidelity_enhancer(mini.to(self.device)).cpu())
        return (x_new_l, x_new_h, x_new), torch.cat(out)

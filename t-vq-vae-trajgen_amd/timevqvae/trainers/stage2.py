"""Stage2 (MaskGIT prior) trainer — the reference trainers/stage2.py contract without
Lightning.  The validation-time sampling metrics (FID/IS via ROCKET, stage2.py:70-110)
are evaluation, out of the hot-path scope; X_train/X_test/fcn args are accepted."""
import torch
import torch.nn as nn

from ..hip.optim import FusedAdamW
from ..models.maskgit import MaskGIT
from ..utils import linear_warmup_cosine_annealingLR
from ..utils.checkpoint import adapt_state_dict, read_state_dict, save_checkpoint


class Stage2(nn.Module):
    def __init__(self, stage1_ckpt_fname: str, fcn_ckpt_fname: str, input_length: int,
                 in_channels: int, n_classes: int, X_train=None, X_test=None, config: dict = None,
                 device=None, feature_extractor_type: str = "supervised_fcn", **kwargs):
        super().__init__()
        self.config = config
        self.maskgit = MaskGIT(stage1_ckpt_fname=stage1_ckpt_fname, input_length=input_length,
                               in_channels=in_channels, config=config, n_classes=n_classes,
                               **config["MaskGIT"], **kwargs)
        self._sched = None
        self._opt = None

    def training_step(self, batch, batch_idx):
        """stage2.py:49-68."""
        x, y = batch
        mask_pred_loss, (loss_l, loss_h) = self.maskgit(x, y)
        if self._sched is not None:
            self._sched.step()
        return {"loss": mask_pred_loss, "mask_pred_loss": mask_pred_loss,
                "mask_pred_loss_l": loss_l, "mask_pred_loss_h": loss_h}

    def forward_backward(self, batch, one):
        """training_step + the backward of its loss, each prior backpropagated from its own
        loss on its own stream (MaskGIT.forward_backward: the same gradients as
        loss.backward()).  `one`: a cached 0-dim ones tensor.  Returns a callable building
        training_step's dict; call it after the streams are joined."""
        x, y = batch
        total = self.maskgit.forward_backward(x, y, one)
        if self._sched is not None:
            self._sched.step()

        def out():
            loss, (loss_l, loss_h) = total()
            return {"loss": loss, "mask_pred_loss": loss, "mask_pred_loss_l": loss_l,
                    "mask_pred_loss_h": loss_h}
        return out

    @torch.no_grad()
    def validation_step(self, batch, batch_idx):
        self.eval()
        x, y = batch
        mask_pred_loss, (loss_l, loss_h) = self.maskgit(x, y)
        return {"loss": mask_pred_loss, "mask_pred_loss_l": loss_l, "mask_pred_loss_h": loss_h}

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True,
                             weights_only=True, **kwargs):
        """Lightning-style loader as generation/sampler.py:76-90 calls it: the constructor
        arguments come as kwargs (the reference saves no hyper-parameters), the frozen
        stage1 is read from `stage1_ckpt_fname` by MaskGIT (maskgit.py:52-59), then every
        tensor of `stage2.ckpt` (stage1 copies included) is loaded, x-transformers key
        drift adapted (utils/checkpoint.py)."""
        sd = read_state_dict(checkpoint_path, map_location, weights_only)
        kwargs.setdefault("stage1_ckpt_fname", None)
        kwargs.setdefault("fcn_ckpt_fname", None)
        model = cls(**kwargs)
        model.load_state_dict(adapt_state_dict(sd, model), strict=strict)
        return model

    def save_checkpoint(self, path, **extra):
        save_checkpoint(self, path, **extra)

    def configure_optimizers(self):
        """stage2.py:112-119 (frozen stage1 parameters carry no grad and are skipped)."""
        opt = FusedAdamW(self.parameters(), lr=self.config["exp_params"]["lr"])
        sch = linear_warmup_cosine_annealingLR(opt, self.config["trainer_params"]["max_steps"]["stage2"],
                                               self.config["exp_params"]["linear_warmup_rate"])
        self._opt, self._sched = opt, sch
        return {"optimizer": opt, "lr_scheduler": sch}

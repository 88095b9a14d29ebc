"""Stage3 (FidelityEnhancer) trainer -- the reference trainers/stage3.py contract without
Lightning (its validation plots and running metrics are evaluation, outside the path).

  training_step (stage3.py:197-231): frozen MaskGIT stage1 encoders with stochastic VQ
    (svq_temp = the FE's tau) -> LF / HF token indices -> decode -> x' (detached) ->
    FidelityEnhancer (training mode: HIP forward + backward, models/fidelity_enhancer.py)
    -> L1(FE(x'), x); percept_loss_weight > 0 (MiniRocket perceptual loss) is not on the
    path and raises.
  search_optimal_tau (stage3.py:88-181): unconditional samples vs. x' re-encoded at each tau
    of fidelity_enhancer.tau_search_rng; FID on the device (evaluation.calculate_fid after
    the reference's IsolationForest outlier removal); tau = argmin FID.
  configure_optimizers (stage3.py:362-369): AdamW (FusedAdamW: only the FE has gradients)
    + linear warm-up / cosine LR schedule over trainer_params.max_steps.stage3.
"""
import numpy as np
import torch
import torch.nn as nn

from ..evaluation import calculate_fid
from ..hip import rng
from ..hip.loss import l1_loss
from ..hip.optim import FusedAdamW
from ..models import FidelityEnhancer
from ..utils import freeze, linear_warmup_cosine_annealingLR, remove_outliers
from .stage2 import Stage2


class Stage3(nn.Module):
    def __init__(self, stage1_ckpt_fname, stage2_ckpt_fname, fcn_ckpt_fname, input_length: int,
                 in_channels: int, n_classes: int, X_train=None, X_test=None, config: dict = None,
                 device=None, feature_extractor_type: str = "supervised_fcn", stage2=None):
        """As the reference (stage3.py:17-86); `stage2` (an already-built Stage2) replaces
        loading `stage2_ckpt_fname` when given."""
        super().__init__()
        self.config = config
        self.in_channels = in_channels
        self.n_fft = config["VQ-VAE"]["n_fft"]
        self.tau_search_rng = config["fidelity_enhancer"]["tau_search_rng"]
        self.fidelity_enhancer = FidelityEnhancer(input_length=input_length,
                                                  in_channels=in_channels, config=config)
        if stage2 is None:
            stage2 = Stage2.load_from_checkpoint(
                stage2_ckpt_fname, stage1_ckpt_fname=stage1_ckpt_fname,
                fcn_ckpt_fname=fcn_ckpt_fname, input_length=input_length,
                in_channels=in_channels, n_classes=n_classes, config=config,
                map_location="cpu")
        freeze(stage2)
        stage2.eval()
        self.maskgit = stage2.maskgit
        self.encoder_l = self.maskgit.encoder_l
        self.decoder_l = self.maskgit.decoder_l
        self.vq_model_l = self.maskgit.vq_model_l
        self.encoder_h = self.maskgit.encoder_h
        self.decoder_h = self.maskgit.decoder_h
        self.vq_model_h = self.maskgit.vq_model_h
        self.percept_loss_weight = config["fidelity_enhancer"].get("percept_loss_weight", 0.0)
        if feature_extractor_type not in ("supervised_fcn", "rocket"):
            raise ValueError(f"unknown feature_extractor_type {feature_extractor_type!r}")
        self.feature_extractor_type = feature_extractor_type
        # The reference's Metrics draws its ROCKET kernels when the model is built
        # (evaluation/metrics.py:89-93, from stage3.py:73-83), so the np.random state they
        # come from is the one at construction, not at the tau search.
        self._rocket_fn = (_rocket_features(input_length, device or "cuda")
                           if feature_extractor_type == "rocket" else None)
        self._sched = None
        self._opt = None

    # ------------------------------------------------------------------ tau search
    @torch.no_grad()
    def search_optimal_tau(self, X_train: np.ndarray, device, n_samples: int = 1024,
                           batch_size: int = 32, feature_fn=None):
        """stage3.py:88-181.  feature_fn(X (n, c, l) float64) -> Z (n, d) overrides the
        extractor.  Without it the extractor follows feature_extractor_type as the reference's
        Metrics.extract_feature_representations does (metrics.py:107-127): 'rocket' uses the
        kernels drawn at construction; 'supervised_fcn' needs the pretrained FCN, which is
        not on this path, so it raises instead of silently using another feature space."""
        if feature_fn is None:
            if self.feature_extractor_type != "rocket":
                raise NotImplementedError(
                    "search_optimal_tau with feature_extractor_type='supervised_fcn' needs the "
                    "pretrained FCN extractor (not on the HIP path): pass feature_fn, or build "
                    "Stage3 with feature_extractor_type='rocket'")
            feature_fn = self._rocket_fn
        maskgit = self.maskgit.to(device)
        n_iters = -(-n_samples // batch_size)
        xhat = []
        for _ in range(n_iters):
            s_l, s_h = maskgit.iterative_decoding(num=batch_size, device=device, class_index=None)
            xhat.append((maskgit.decode_token_ind_to_timeseries(s_l, "lf")
                         + maskgit.decode_token_ind_to_timeseries(s_h, "hf")).cpu())
        Zhat = feature_fn(torch.cat(xhat).numpy().astype(float))
        fids = []
        for tau in self.tau_search_rng:
            xprime = []
            for i in range(-(-X_train.shape[0] // batch_size)):
                x = torch.from_numpy(X_train[i * batch_size:(i + 1) * batch_size]).float().to(device)
                _, sl = maskgit.encode_to_z_q(x, self.encoder_l, self.vq_model_l, svq_temp=tau)
                _, sh = maskgit.encode_to_z_q(x, self.encoder_h, self.vq_model_h, svq_temp=tau)
                xprime.append((maskgit.decode_token_ind_to_timeseries(sl, "lf")
                               + maskgit.decode_token_ind_to_timeseries(sh, "hf")).cpu())
            Zp = feature_fn(torch.cat(xprime).numpy().astype(float))
            fids.append(float(calculate_fid(remove_outliers(Zhat), remove_outliers(Zp))))
        self.tau_fids = dict(zip(self.tau_search_rng, fids))
        optimal_tau = self.tau_search_rng[int(np.argmin(fids))]
        self.fidelity_enhancer.tau = torch.tensor(optimal_tau).float().to(self.fidelity_enhancer.tau.device)
        return optimal_tau

    # ------------------------------------------------------------------ losses
    def _fidelity_enhancer_loss_fn(self, x, sprime_l, sprime_h):
        """stage3.py:193-210."""
        xprime = (self.maskgit.decode_token_ind_to_timeseries(sprime_l, "lf")
                  + self.maskgit.decode_token_ind_to_timeseries(sprime_h, "hf")).detach()
        xhat = self.fidelity_enhancer(xprime)
        recons_loss = l1_loss(xhat, x)
        return recons_loss, (xprime, xhat)

    def _perceptual_loss_fn(self, x, xprime_R):
        """stage3.py:212-221: 0 unless percept_loss_weight > 0 (MiniRocket, not on the path)."""
        if self.percept_loss_weight > 0:
            raise NotImplementedError("percept_loss_weight > 0 (MiniRocket) is not on the HIP path")
        return 0.0

    def _step_losses(self, x):
        tau = float(self.fidelity_enhancer.tau)
        _, sprime_l = self.maskgit.encode_to_z_q(x, self.encoder_l, self.vq_model_l, svq_temp=tau)
        _, sprime_h = self.maskgit.encode_to_z_q(x, self.encoder_h, self.vq_model_h, svq_temp=tau)
        fe_loss, (xprime, xprime_R) = self._fidelity_enhancer_loss_fn(x, sprime_l, sprime_h)
        percept_loss = self._perceptual_loss_fn(x, xprime_R)
        loss = fe_loss + percept_loss
        return {"loss": loss, "fidelity_enhancer_loss": fe_loss, "percept_loss": percept_loss}

    def training_step(self, batch, batch_idx):
        """stage3.py:223-256: everything frozen in eval mode, the FE in training mode."""
        self.eval()
        self.fidelity_enhancer.train()
        x, _ = batch
        rng.advance(x.device)  # fresh dropout masks for this step
        out = self._step_losses(x.float())
        if self._sched is not None:
            self._sched.step()
        return out

    @torch.no_grad()
    def validation_step(self, batch, batch_idx):
        """stage3.py:258-263 (the losses; sampling plots and running metrics are not run)."""
        self.eval()
        x, _ = batch
        return self._step_losses(x.float())

    def configure_optimizers(self):
        """stage3.py:362-369: AdamW over the (trainable) parameters + warm-up cosine LR."""
        opt = FusedAdamW(self.parameters(), lr=self.config["exp_params"]["lr"])
        sch = linear_warmup_cosine_annealingLR(
            opt, self.config["trainer_params"]["max_steps"]["stage3"],
            self.config["exp_params"]["linear_warmup_rate"])
        self._opt, self._sched = opt, sch
        return {"optimizer": opt, "lr_scheduler": sch}


def _rocket_features(input_length, device, num_kernels=1000):
    """The reference's `rocket` feature extractor (evaluation/metrics.py:113-117): ROCKET
    features of channel 0 (on the device), each row L2-normalised in float32."""
    from ..evaluation import DeviceKernels, apply_kernels_device, generate_kernels
    dk = DeviceKernels(generate_kernels(input_length, num_kernels), device)

    def fn(X):
        x0 = torch.from_numpy(np.ascontiguousarray(np.asarray(X)[:, 0, :], dtype=np.float64))
        z = apply_kernels_device(x0.to(device), dk).float()
        return torch.nn.functional.normalize(z, p=2, dim=-1).cpu().numpy()
    return fn

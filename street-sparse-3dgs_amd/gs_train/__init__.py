"""gs_train -- the device work of one Street-sparse-3DGS training iteration around the rasterizer
(SURVEY.md 8(a) row H, 8(f) rows 1-2), on the gfx950 kernels of csrc/train.hip:

  loss.l1_ssim / loss.photo_loss   fused L1 + SSIM forward/backward (utils/loss_utils.py)
  optim.Adam                       fused sparse Adam, drop-in for scene/OurAdam.Adam
  exposure.apply_exposure          per-image exposure affine + clamp (gaussian_renderer/__init__.py:115-120)
  densify.add_densification_stats  train_single.py:193-194 + scene/gaussian_model.py:780-793
  activations.activate             exp / normalize / sigmoid getters fwd+bwd in one launch each
  activations.shrink_scales        the per-step shrink of over-large Gaussians (train_single.py:235-241)
  harness.TrainStep                one train_single.py inner-loop iteration (the "train-step ms")
  native_step.NativeTrainStep      the same iteration as one native call (gsr_train_step)
  synthetic                        seeded synthetic scenes / cameras
"""
from .loss import l1_ssim, photo_loss  # noqa: F401
from .optim import Adam  # noqa: F401
from .densify import add_densification_stats  # noqa: F401
from .exposure import apply_exposure  # noqa: F401
from .activations import activate, shrink_scales  # noqa: F401

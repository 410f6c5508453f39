"""Generator / discriminator losses (losses.py of the reference) on encx kernels."""
import torch

from . import ops

MEL_SCALES = tuple(2 ** i for i in range(5, 12))  # losses.py:40, n_fft = 32 .. 2048


def reconstruction_losses(input_wav, output_wav, sample_rate=24000):
    """l_t (losses.py:37) and l_f (losses.py:40-42)."""
    l_t = ops.L1LossFn.apply(input_wav, output_wav)
    l_f = ops.MelLossFn.apply(input_wav, output_wav, sample_rate, 64, MEL_SCALES)
    return l_t, l_f


def total_loss(fmap_real, logits_fake, fmap_fake, input_wav, output_wav, sample_rate=24000):
    """losses.py:4-63. With fmap_real None (generator-only training, config 2) only l_t and l_f
    are returned."""
    l_t, l_f = reconstruction_losses(input_wav, output_wav, sample_rate)
    out = {'l_t': l_t, 'l_f': l_f}
    if fmap_real is None:
        return out
    from .msstftd import adversarial_losses
    l_g, l_feat = adversarial_losses(fmap_real, logits_fake, fmap_fake)
    out['l_g'] = l_g
    out['l_feat'] = l_feat
    return out


def disc_loss(logits_real, logits_fake):
    """losses.py:65-80."""
    from .msstftd import hinge_disc_loss
    return hinge_disc_loss(logits_real, logits_fake)

"""Drop-in module name of the reference's ``ptp_utils.py`` (re-exports p2p_amd.ptp_utils)."""
from p2p_amd.ptp_utils import *  # noqa: F401,F403
from p2p_amd.ptp_utils import (DummyController, diffusion_step, get_time_words_attention_alpha,  # noqa: F401
                               get_word_inds, init_latent, latent2image, register_attention_control,
                               text2image_ldm, text2image_ldm_stable, update_alpha_time_word)

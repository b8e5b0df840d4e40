"""Drop-in module name of the reference's ``seq_aligner.py`` (re-exports p2p_amd.seq_aligner)."""
from p2p_amd.seq_aligner import *  # noqa: F401,F403
from p2p_amd.seq_aligner import (ScoreParams, get_aligned_sequences, get_mapper, get_matrix,  # noqa: F401
                                 get_refinement_mapper, get_replacement_mapper, get_replacement_mapper_,
                                 get_traceback_matrix, get_word_inds, global_align)

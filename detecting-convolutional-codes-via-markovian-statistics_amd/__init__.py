"""MI355X-native Monte-Carlo relative-Viterbi-metric detector.

Drop-in for the hot path of So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics
(Pd_plotter.run_experiment and the functions beneath it), running on gfx950
through libcvd.so (include/cvd.h).  See DESIGN.md.
"""
from ._lib import CvdError, lib, PATH_AUTO, PATH_TABLE, PATH_EXPLICIT, PATH_EXPLICIT_GENERIC, PATH_EXPLICIT_ORBIT, PATH_EXPLICIT_BUTTERFLY, KERNEL_NAMES  # noqa: F401
from .codes import Code, EXAMPLE_CODES, CONFIG_CODES, octal_to_taps  # noqa: F401
from .detector import (  # noqa: F401
    DEFAULTS, N_SPECTRUM_BY_M, Detector, Model, run_experiment, learn_P1_empirical,
    enumerate_markov_states_allzero, build_trellis, branch_output_and_next_state,
    viterbi_metric_step, simulate_markov_sequence, log_likelihood_ratio, grid_tag, LEARN_TAG,
    enumerate_states_device,
)
from .parity import (  # noqa: F401
    parse_poly_token, build_parity_system, nullspace_mod2, parity_vector_to_equation, parity_vectors,
    template_of, default_template, parity_detect, parity_satisfaction_fraction, parity_detector,
    parity_experiment,
)
from .exponent import (  # noqa: F401
    TransitionTensor, learn_transition_tensor, chernoff_rhos, compute_error_exponent, spectral_radius,
    fit_error_exponent, EXPONENT_TAG,
)

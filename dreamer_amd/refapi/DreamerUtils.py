"""Reference module name `DreamerUtils` (drop-in); see INTEGRATION.md."""
from dreamer_amd.utils import (_sanitize_for_save, bernoulli_log_probability, gaussian_log_probability,  # noqa: F401
                              kullback_leibler_divergence_between_gaussians, symexp, symlog, symlog_np, to_twohot)

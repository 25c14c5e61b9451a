"""DreamerUtils (reference DreamerUtils.py): the helpers the reference's
callers import.  symlog/symexp/two-hot are also inlined in the HIP kernels
(common.h, ops.hip); these torch versions serve the world-model training step
and user code."""
import numpy as np
import torch


def gaussian_log_probability(x, mu, sigma):  # DreamerUtils.py:4-10
    return torch.distributions.Normal(loc=mu, scale=sigma).log_prob(x)


def bernoulli_log_probability(p, k):  # DreamerUtils.py:12-16
    pc = torch.clamp(p, min=1e-8, max=1.0 - 1e-8)
    return k * torch.log(pc) + (1 - k) * torch.log(1 - pc)


def kullback_leibler_divergence_between_gaussians(mu_1, sigma_1, mu_2, sigma_2):  # DreamerUtils.py:18-27
    v1, v2 = torch.square(sigma_1), torch.square(sigma_2)
    return torch.log(sigma_2 / sigma_1) + ((v1 + torch.square(mu_1 - mu_2)) / (2 * v2)) - 0.5


def symlog(x):  # DreamerUtils.py:29-30
    return torch.sign(x) * torch.log(1.0 + torch.abs(x))


def symlog_np(x):  # DreamerUtils.py:32-33
    return np.sign(x) * np.log(1.0 + np.abs(x))


def symexp(x):  # DreamerUtils.py:35-37
    x = torch.clamp(x, -20.0, 20.0)
    return torch.sign(x) * (torch.exp(torch.abs(x).float()) - 1.0)


def to_twohot(value, buckets):  # DreamerUtils.py:39-50
    v = torch.clamp(value, min=buckets.min(), max=buckets.max())
    lo = torch.clamp(torch.searchsorted(buckets, v, right=True) - 1, max=len(buckets) - 2)
    w = (v - buckets[lo]) / (buckets[lo + 1] - buckets[lo] + 1e-8)
    out = torch.zeros(value.shape[:-1] + (buckets.shape[0],), dtype=torch.float32, device=value.device)
    out = torch.scatter(out, -1, lo, 1.0 - w)
    return torch.scatter(out, -1, lo + 1, w)


def _sanitize_for_save(data_list):  # DreamerUtils.py:52-63 (training_logs.npz schema)
    out = []
    for item in data_list:
        if isinstance(item, torch.Tensor):
            out.append(item.detach().cpu().item())
        elif isinstance(item, list):
            out.append([x.detach().cpu().item() if isinstance(x, torch.Tensor) else x for x in item])
        else:
            out.append(item)
    return np.array(out)

"""Glue between the reference-shaped nn.Modules and libdreamer_hip: packs
parameters (in PyTorch's own layout, no copies) into the C structs, owns
per-device workspaces and the Philox RNG state."""
import os
import threading

import torch

from . import _lib as L

_tls = threading.local()


def linear(mod):
    """dr_linear for an nn.Linear / nn.LayerNorm (None -> NULL)."""
    if mod is None:
        return L.dr_linear(None, None)
    return L.dr_linear(L.ptr(mod.weight), L.ptr(mod.bias))


def mlp3(seq):
    """dr_mlp3 for Sequential(Linear, LN, SiLU, Linear, LN, SiLU, Linear)."""
    return L.dr_mlp3(linear(seq[0]), linear(seq[1]), linear(seq[3]), linear(seq[4]), linear(seq[6]))


def linear_grad(mod):
    """dr_linear pointing at the .grad tensors of an nn.Linear / LayerNorm / conv."""
    return L.dr_linear(L.ptr(mod.weight.grad), L.ptr(mod.bias.grad))


def mlp3_grad(seq):
    return L.dr_mlp3(linear_grad(seq[0]), linear_grad(seq[1]), linear_grad(seq[3]), linear_grad(seq[4]),
                     linear_grad(seq[6]))


def flat_linear(flat, offsets, key_w, key_b):
    base = flat.data_ptr()
    return L.dr_linear(base + 4 * offsets[key_w], base + 4 * offsets[key_b])


class Workspace:
    """Grow-only scratch buffers on one device, keyed by name.

    DREAMER_WS_POISON=all (or a comma list of names) fills new buffers with
    0xFF bytes (f32 NaN): a kernel that reads scratch it has not written
    then poisons its outputs (tests/test_gpu_api.py workspace test)."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

    def get(self, name, nbytes):
        nbytes = max(int(nbytes), 256)
        b = self.bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            poison = os.environ.get("DREAMER_WS_POISON", "")
            if poison == "all" or name in poison.split(","):
                b.fill_(0xFF)
            self.bufs[name] = b
        return b


_ws = {}


def workspace(device):
    key = torch.device(device).index or 0
    if key not in _ws:
        _ws[key] = Workspace(torch.device("cuda", key))
    return _ws[key]


class Rng:
    """Device Philox state {seed, offset} (uint64 x2).  The seed is drawn from
    torch's CPU generator so torch.manual_seed controls it.

    Two generators per device: `rng(dev)` is the engine's (its call sites use
    fixed stream ids, WARM_STREAM / DREAM_STREAM in engine.py), and
    `adhoc(dev)` serves the one-off API calls (acting, encode, observe_step,
    the world-model step) with a different seed, so the two can never draw the
    same variates.  Each ad-hoc call gets a fresh stream id counter << 17 (a
    call's kernels add at most 65536 + a step index to it); when the 14-bit
    counter wraps, the device offset is advanced so ids are never reused."""

    STREAM_SHIFT = 17
    COUNTER_MASK = (1 << 14) - 1

    def __init__(self, device, salt=0):
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item()) ^ salt
        self.state = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        self.counter = 0
        self.salt = salt

    def reseed(self, seed):
        self.state.copy_(torch.tensor([seed, 0], dtype=torch.int64))
        self.counter = 0

    def noise(self, row0=0):
        if _override and self.salt:
            q, eps = _override[-1]
            return L.dr_noise(L.ptr(q) if q is not None else None, L.ptr(eps) if eps is not None else None,
                              self.state.data_ptr(), row0, 0)
        self.counter = (self.counter + 1) & self.COUNTER_MASK
        if self.counter == 0:
            L.call("dr_rng_advance", self.state.data_ptr(), 1, stream())
            self.counter = 1
        return L.dr_noise(None, None, self.state.data_ptr(), row0, self.counter << self.STREAM_SHIFT)


_rngs = {}
_adhoc = {}


def rng(device):
    """The engine's generator (fixed per-call-site stream ids)."""
    key = torch.device(device).index or 0
    if key not in _rngs:
        _rngs[key] = Rng(torch.device("cuda", key))
    return _rngs[key]


def adhoc(device):
    """The generator of one-off API calls (see Rng)."""
    key = torch.device(device).index or 0
    if key not in _adhoc:
        _adhoc[key] = Rng(torch.device("cuda", key), salt=0x5DEECE66D)
    return _adhoc[key]


_override = []


class noise_override:
    """Parity mode for the one-off API calls (SURVEY §5 "noise: explicit"):
    inside the block every ad-hoc draw reads the given variates instead of
    Philox -- q: Exp(1) [steps][rows*R][C] for categorical samples, eps:
    N(0,1) [steps][rows][A] for actor samples (device tensors; the caller
    keeps them alive).  The engine's own draws are not affected."""

    def __init__(self, q=None, eps=None):
        self.q, self.eps = q, eps

    def __enter__(self):
        _override.append((self.q, self.eps))
        return self

    def __exit__(self, *exc):
        _override.pop()
        return False


def explicit_noise(q=None, eps=None, device=None):
    """dr_noise reading caller-supplied variates (parity mode)."""
    st = rng(device).state.data_ptr() if device is not None else None
    return L.dr_noise(L.ptr(q) if q is not None else None, L.ptr(eps) if eps is not None else None, st, 0, 0)


def stream():
    return L.stream_ptr()


def needs_torch_grad(*mods):
    """True when autograd through these modules' parameters is requested
    (the world-model training step, which stays PyTorch-ROCm this round)."""
    if not torch.is_grad_enabled():
        return False
    return any(p.requires_grad for m in mods for p in m.parameters())

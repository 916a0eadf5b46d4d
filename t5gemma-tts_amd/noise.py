"""Parity-mode sampling noise: the reference's torch.multinomial draws, made on the GPU.

The reference samples each step with ``torch.multinomial(p, 1)`` on CPU
(hf_export/modeling_t5gemma_voice.py:133-138), i.e. V exponential variates from torch's
global CPU generator -- an MT19937 engine (SURVEY a14' step 6; csrc/noise.hip holds the
restatement). This module moves a generator's state to and from the 625-word form the
device kernel takes (624 state words + outputs already consumed of that state) and runs
the kernel: one MT19937 stream per row, written raw to HBM, read by the engine's sampler.

torch's CPUGeneratorImplState byte layout (torch 2.10, ``Generator.get_state()``, 5056
bytes): uint64 the_initial_seed | int32 left | int32 seeded | uint64 next |
uint64 state[624] | double normal_x, normal_y, normal_rho | int32 normal_is_valid |
float next_float_normal_sample | bool valid. The engine outputs ``state[next++]`` after a
twist when ``--left`` reaches 0, so the consumed position is ``625 - left``.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib

MT_N = 624
MT_W = MT_N + 1
_STATE_BYTES = 5056
_OFF_LEFT, _OFF_NEXT, _OFF_STATE = 8, 16, 24


def _state_bytes(g: torch.Generator) -> np.ndarray:
    st = g.get_state().numpy()
    if st.size != _STATE_BYTES:
        raise RuntimeError(f"unexpected torch CPU generator state size {st.size} (torch 2.10 layout: {_STATE_BYTES})")
    return st


def mt_words(src: Union[int, torch.Generator]) -> np.ndarray:
    """[625] uint32: the MT19937 words + consumed position of a torch CPU generator (or of
    ``torch.manual_seed(src)`` for an int)."""
    g = src if isinstance(src, torch.Generator) else torch.Generator().manual_seed(int(src))
    st = _state_bytes(g)
    left = int(st[_OFF_LEFT:_OFF_LEFT + 4].view(np.int32)[0])
    words = st[_OFF_STATE:_OFF_STATE + 8 * MT_N].view(np.uint64).astype(np.uint32)
    out = np.empty(MT_W, np.uint32)
    out[:MT_N] = words
    out[MT_N] = 625 - left
    return out


def set_generator(g: torch.Generator, words: np.ndarray) -> None:
    """Put a [625] snapshot (words + consumed position) back into torch generator ``g``
    (the seed and the normal-sampling caches are kept)."""
    st = _state_bytes(g).copy()
    pos = int(words[MT_N])
    if not 1 <= pos <= MT_N:
        raise ValueError(f"MT19937 snapshot position {pos} outside 1..624")
    st[_OFF_LEFT:_OFF_LEFT + 4] = np.array([625 - pos], np.int32).view(np.uint8)
    st[_OFF_NEXT:_OFF_NEXT + 8] = np.array([pos], np.uint64).view(np.uint8)
    st[_OFF_STATE:_OFF_STATE + 8 * MT_N] = words[:MT_N].astype(np.uint64).view(np.uint8)
    g.set_state(torch.from_numpy(st))


class DeviceNoise:
    """Raw MT19937 outputs of B rows for ``steps`` sampler steps, on the device.

    Buffers are kept between calls (a fixed per-row stride of ``cap_steps`` steps), so the
    pointer the engine's captured graphs read stays the same."""

    def __init__(self, V: int, device):
        self.V = V
        self.device = torch.device(device)
        self.raw: Optional[torch.Tensor] = None
        self.snap: Optional[torch.Tensor] = None
        self.cap_rows = self.cap_steps = 0
        self.event = None

    def ensure(self, rows: int, cap_steps: int) -> None:
        if self.raw is None or rows > self.cap_rows or cap_steps != self.cap_steps:
            self.raw = None
            self.raw = torch.empty(rows, cap_steps * 2 * self.V, dtype=torch.int32, device=self.device)
            self.cap_rows, self.cap_steps = rows, cap_steps

    def generate(self, sources: Sequence[Union[int, torch.Generator]], steps: int, cap_steps: int,
                 snapshots: bool, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Launch the per-row streams (``steps`` steps each) on ``stream`` (default: a side
        stream; ``self.event`` then marks completion)."""
        B = len(sources)
        if steps > cap_steps:
            raise ValueError(f"{steps} noise steps > capacity {cap_steps}")
        self.ensure(max(B, self.cap_rows), cap_steps)
        init = torch.from_numpy(np.stack([mt_words(s) for s in sources]).view(np.int32)).to(self.device)
        V2 = 2 * self.V
        self.snap = torch.empty(B, steps + 1, MT_W, dtype=torch.int32, device=self.device) if snapshots else None
        side = stream or torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            _lib.check(_lib.lib().t5g_mt_stream(
                C.c_void_p(init.data_ptr()), B, steps * V2, cap_steps * V2, C.c_void_p(self.raw.data_ptr()),
                V2, steps + 1, C.c_void_p(self.snap.data_ptr()) if snapshots else None,
                C.c_void_p(side.cuda_stream)), "mt_stream")
            init.record_stream(side)
            self.event = torch.cuda.Event()
            self.event.record(side)

    def q_row(self, b: int, step: int) -> torch.Tensor:
        """bf16 [V] (host): the draws of row b at sampler step ``step`` (host-resolved steps)."""
        V2 = 2 * self.V
        q = torch.empty(self.V, dtype=torch.bfloat16, device=self.device)
        src = self.raw[b, step * V2:(step + 1) * V2]
        _lib.check(_lib.lib().t5g_mt_exponential(C.c_void_p(src.data_ptr()), self.V, C.c_void_p(q.data_ptr()),
                                                 C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "mt_exponential")
        return q.cpu()

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        if self.event is not None:
            (stream or torch.cuda.current_stream(self.device)).wait_event(self.event)

    def advance_generators(self, gens: Sequence[torch.Generator], steps_used: Sequence[int]) -> None:
        """Leave each generator where the reference's loop leaves torch's: after exactly
        ``steps_used[b]`` multinomial calls (the snapshot of that step boundary)."""
        if self.snap is None:
            raise RuntimeError("noise generated without snapshots")
        idx = torch.tensor(list(steps_used), dtype=torch.long, device=self.device)
        rows = self.snap[torch.arange(len(gens), device=self.device), idx].cpu().numpy().view(np.uint32)
        for g, w in zip(gens, rows):
            set_generator(g, w)


def host_q(raw_pairs: np.ndarray) -> np.ndarray:
    """Reference restatement of the draw (test helper): raw uint32 [..., 2] -> fp32 q
    (the bf16 value), torch's uniform_real_distribution<double> + -log1p(-u)."""
    r = (raw_pairs[..., 0].astype(np.uint64) << np.uint64(32)) | raw_pairs[..., 1].astype(np.uint64)
    u = (r & np.uint64((1 << 53) - 1)).astype(np.float64) * 2.0 ** -53
    x = (-np.log1p(-u)).astype(np.float32)
    return torch.from_numpy(x).to(torch.bfloat16).float().numpy()

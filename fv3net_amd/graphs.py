"""Launch-bound steps captured into HIP graphs.

A prognostic step on one rank's band is a handful of short kernels (the fused predict,
the limiter/diagnostics epilogue, the row partials, the level counts, the fold), each
behind a Python call that marshals its arguments through ctypes.  At C96 over 8 GPUs
(6,912 columns per rank) the kernels take ~45 us and the host-side launches ~120 us, so
the step is bound by the host, not the GPU.  ``StepGraph`` records such a step once on
the current stream into a hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and
replays it with one ``hipGraphLaunch`` per step.

What a captured step must satisfy (the workloads in ``workloads.py`` are written so):
  * every launch goes to the current stream (the C-ABI calls take
    ``torch.cuda.current_stream()``, which is the capture stream inside the capture);
  * its inputs and outputs are fixed device buffers: a value carried from one step to
    the next (e.g. the accumulated precipitation) is copied back into its input buffer
    inside the step, since a replay re-reads the addresses recorded at capture;
  * no host synchronisation or host reads inside it; collectives stay outside (the
    caller runs them between graphs).
The first call of the wrapped function must already have run eagerly (lazy native
initialisation, model upload, occupancy caches): ``StepGraph`` is built after it.
"""
from typing import Callable

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None


class StepGraph:
    """``fn`` captured on first call, replayed on every call; returns ``fn``'s outputs
    as captured (tensors the replay rewrites in place)."""

    def __init__(self, fn: Callable):
        self.fn = fn
        self.graph = None
        self.out = None

    def capture(self):
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.fn()
        self.graph = g

    def __call__(self):
        if self.graph is None:
            self.capture()  # records only: the replay below runs the step
        self.graph.replay()
        return self.out

"""The remap entry points under the reference build's arithmetic (``exact=True``).

The parity tests that assert bit-identity with the flang-compiled mappm.f90 (golden
vectors), with oracle/coarsen.py / oracle/restarts.py bitwise, or between kernels of the
exact path import the remap API from here.  The product default is the tolerance
contract (``exact=False``, csrc/mappm_core.h); tests/test_remap_fast.py holds that path
to its bounds against the same references."""
import functools

from fv3net_amd import coarsen as _coarsen
from fv3net_amd import mappm as _mappm
from fv3net_amd import restarts as _restarts

mappm_device = functools.partial(_mappm.mappm_device, exact=True)
mappm_device_multi = functools.partial(_mappm.mappm_device_multi, exact=True)
coarsen_on_pressure = functools.partial(_coarsen.coarsen_on_pressure, exact=True)
coarsen_edges_on_pressure = functools.partial(_coarsen.coarsen_edges_on_pressure, exact=True)
regrid_vertical = functools.partial(_coarsen.regrid_vertical, exact=True)
coarsen_restarts_on_pressure = functools.partial(_restarts.coarsen_restarts_on_pressure, exact=True)


class MappmPlan(_mappm.MappmPlan):
    def __init__(self, *args, exact=True, **kwargs):
        super().__init__(*args, exact=exact, **kwargs)


class MappmMultiPlan(_mappm.MappmMultiPlan):
    def __init__(self, *args, exact=True, **kwargs):
        super().__init__(*args, exact=exact, **kwargs)


def __getattr__(name):  # everything else unchanged (mappm, TOA_PRESSURE, weighted_block_average, ...)
    for m in (_mappm, _coarsen, _restarts):
        if hasattr(m, name):
            return getattr(m, name)
    raise AttributeError(name)

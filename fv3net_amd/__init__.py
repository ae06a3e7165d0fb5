"""fv3net_amd — MI355X-native build of fv3net's per-timestep ML-physics hot path.

Scope: the column-wise ``fv3fit.Predictor.predict`` issued by the
prognostic run's ML stepper, the ``external/mappm`` vertical remap and the
``vcm.cubedsphere`` stack/unstack + pressure-level block coarsening that feed it.
All arithmetic runs in the HIP library ``fv3net_amd/_lib/libfv3net_amd.so``
(C ABI: ``include/fv3net_amd.h``); there is no CPU fallback.
"""
__version__ = "0.1.0"

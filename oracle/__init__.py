"""ORACLE package — test infrastructure only.

Nothing in ``fv3net_amd`` imports, links or executes anything under ``oracle/``.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and only as the checker / CPU baseline, never as the product.

Contents (each function cites the reference file:line it restates):

* ``mappm``    — ctypes wrappers for the C restatement (``mappm_oracle.c``) and for
                 the reference Fortran compiled as-is (``_ref/libmappm_ref.so``).
* ``dense``    — numpy restatement of the fv3fit DenseModel predict graph.
* ``coarsen``  — numpy restatement of vcm.cubedsphere block average / upsample,
                 pressure_at_interface and the area-weighted pressure regrid.
* ``stacking`` — numpy restatement of fv3fit stack / unstack index mapping.
"""

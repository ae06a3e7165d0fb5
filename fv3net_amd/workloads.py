"""Synthetic workloads of BASELINE.json's configs, shared by
bench.py, __graft_entry__.smoke() and the tests.  Inputs are created directly in
HBM (no host round trip inside timed regions)."""
import dataclasses
from typing import List, Optional

import numpy as np

from .dense import DenseColumnModel, DenseModelConfig
from .plan import LaunchPlan

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

NZ = 79
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, dense f32 MFMA (= vector) peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md, dense bf16 MFMA peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak
N_CU = 256             # MI355X compute units (8 XCDs x 32)


def c_columns(res: int, ntile: int = 6) -> int:
    return ntile * res * res


def dense_2x256_config() -> DenseModelConfig:
    """config #2: DenseModel width 256, depth 3 (two hidden layers), T/q -> dQ1/dQ2."""
    return DenseModelConfig(
        input_variables=["air_temperature", "specific_humidity"],
        output_variables=["dQ1", "dQ2"],
        in_nz=[NZ, NZ], out_nz=[NZ, NZ], width=256, depth=3,
    )


def synthetic_state(res: int, seed: int, device, ntile: int = 6):
    """T ~ N(260, 15) K, q ~ U(0, 0.02) kg/kg, (tile, z, y, x) float32 on device."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    shape = (ntile, NZ, res, res)
    T = torch.randn(shape, generator=g, device=device) * 15.0 + 260.0
    q = torch.rand(shape, generator=g, device=device) * 0.02
    return T, q


@dataclasses.dataclass
class DenseWorkload:
    model: DenseColumnModel
    inputs: List
    outputs: List
    ncol: int
    flops_per_column: int
    bytes_per_column: int

    _bound: object = None

    def step(self):
        if self._bound is None:
            self._bound = self.model.bind(self.inputs, level_axes=[1, 1], outputs=self.outputs, out_level_axis=1)
        else:
            self._bound()


def make_dense_workload(res: int, seed: int = 0, device=None, model: Optional[DenseColumnModel] = None,
                        precision: Optional[str] = None):
    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    T, q = synthetic_state(res, seed, device)
    if model is None:
        # normalisation fitted on a sample of the synthetic state (build_model fits on data)
        sample_T = T[0, :, :8, :8].reshape(NZ, -1).T.cpu().numpy()
        sample_q = q[0, :, :8, :8].reshape(NZ, -1).T.cpu().numpy()
        model = DenseColumnModel.random(dense_2x256_config(), seed=1, sample_inputs=[sample_T, sample_q])
    if precision is not None:
        model.precision = precision
    outs = [torch.empty_like(T), torch.empty_like(T)]
    cfg = model.config
    return DenseWorkload(model, [T, q], outs, c_columns(res), cfg.flops_per_column(),
                         4 * (cfg.k_in + cfg.k_out))


@dataclasses.dataclass
class MappmWorkload:
    pe1: object
    q1: object
    pe2: object
    q2: object
    ncol: int
    km: int
    kn: int
    kord: int
    iv: int = 1
    exact: bool = False  # the remap arithmetic (mappm_device)

    @property
    def bytes_per_column(self) -> int:
        return 4 * ((self.km + 1) + self.km + (self.kn + 1) + self.kn)

    plan: object = None

    def step(self):
        from .mappm import MappmPlan

        if self.plan is None:  # prepared once: each step is one C-ABI call
            self.plan = MappmPlan(self.pe1, self.q1, self.pe2, self.iv, self.kord, out=self.q2, exact=self.exact)
        else:
            self.plan()


def make_mappm_workload(ncol: int, km: int = NZ, kn: int = NZ, kord: int = 1, seed: int = 0, device=None,
                        exact: bool = False):
    """Monotone columns: delp ~ D(k) * U(0.99, 1.01) (a 79-level reference profile,
    cf. synth/_restarts.py:36-38), p_out = a neighbour's edges (kn == km) or kn+1
    evenly spaced edges (config #1), shared 300 Pa top."""
    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    base = torch.linspace(200.0, 1800.0, km, device=device)[:, None]
    delp = base * (0.99 + 0.02 * torch.rand((km, ncol), generator=g, device=device))
    top = torch.full((1, ncol), 300.0, device=device)
    pe1 = torch.cat([top, 300.0 + torch.cumsum(delp, 0)])
    if kn == km:
        d2 = base * (0.99 + 0.02 * torch.rand((km, ncol), generator=g, device=device))
        pe2 = torch.cat([top, 300.0 + torch.cumsum(d2, 0)])
    else:
        frac = torch.linspace(0.0, 1.0, kn + 1, device=device)[:, None]
        pe2 = pe1[:1] + frac * (pe1[-1:] - pe1[:1])
    q1 = torch.randn((km, ncol), generator=g, device=device) * 10.0 + 250.0
    q2 = torch.empty((kn, ncol), device=device)
    return MappmWorkload(pe1.contiguous(), q1, pe2.contiguous(), q2, ncol, km, kn, kord, exact=exact)


@dataclasses.dataclass
class CoarsenWorkload:
    """BASELINE config #3: C384 -> C48 (f = 8) pressure-level coarsen of T, 79 levels."""
    delp: object
    area: object
    fields: dict
    factor: int
    ncol_fine: int
    km: int
    exact: bool = False  # the remap arithmetic (coarsen_on_pressure)

    @property
    def bytes_per_column(self) -> float:
        """Algorithmic HBM bytes per FINE column: delp + fields + area read once,
        coarse fields + coarse delp written (636 B + writes)."""
        nf = len(self.fields)
        return 4.0 * (self.km * (1 + nf) + 1) + 4.0 * self.km * (nf + 1) / self.factor ** 2

    def step(self):
        from .coarsen import coarsen_on_pressure

        return coarsen_on_pressure(self.delp, self.area, self.fields, self.factor, exact=self.exact)


def make_coarsen_workload(res: int = 384, factor: int = 8, nfields: int = 1, seed: int = 0, device=None,
                          exact: bool = False):
    """delp ~ D(k) * U(0.99, 1.01) (79-level profile), area ~ U(0.5, 1), T ~ N(250, 10); float32."""
    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    shape = (6, NZ, res, res)
    base = torch.linspace(200.0, 1800.0, NZ, device=device)[None, :, None, None]
    delp = base * (0.99 + 0.02 * torch.rand(shape, generator=g, device=device))
    area = 0.5 + 0.5 * torch.rand((6, res, res), generator=g, device=device)
    fields = {f"f{i}": torch.randn(shape, generator=g, device=device) * 10.0 + 250.0 for i in range(nfields)}
    return CoarsenWorkload(delp, area, fields, factor, 6 * res * res, NZ, exact)


@dataclasses.dataclass
class StepperWorkload:
    """BASELINE config #4 per GPU: one ML-stepper step on a float64 (tile, z, y, x)
    state: float32 model inputs, the fused dense predict of dQ1/dQ2, the fused
    limiter/diagnostics/apply epilogue (in place) and the global means of the 2-D
    diagnostics (area-weighted partials + one all-gather when distributed)."""
    model: DenseColumnModel
    state: dict
    area: object
    dt: float
    ncol: int
    group: object = None
    bound: object = None
    precision: str = "f32"
    _in32: object = None
    _epi: object = None
    _part: object = None
    _plan: object = None

    def _bind(self):
        """Validate and marshal every launch of the step once (the predict, the fused
        epilogue, the area partials): a step is then three C-ABI calls on fixed buffers.
        The state's precipitation becomes the last row of the epilogue's column buffer,
        so the kernel accumulates it in place (it reads a column's total before writing
        the new one)."""
        from .distributed import bind_area_weighted_partials
        from .stepper import BoundEpilogue

        T, q = self.state["air_temperature"], self.state["specific_humidity"]
        if self.precision == "f32":  # the float64 state read in place every step
            self.bound = self.model.bind([T, q], level_axes=[1, 1])
        else:  # the split kernel reads float32: the state is cast into bound buffers each step
            self._in32 = [T.to(torch.float32), q.to(torch.float32)]
            self.bound = self.model.bind(self._in32, level_axes=[1, 1], precision=self.precision)
        dq1, dq2 = self.bound.outputs
        precip = self.state["total_precipitation"]
        column = torch.empty((7, precip.numel()), dtype=precip.dtype, device=precip.device)
        column[6].copy_(precip.reshape(-1))
        self.state["total_precipitation"] = column[6].view(precip.shape)
        self._epi = BoundEpilogue(dq1, dq2, q, self.state["pressure_thickness_of_atmospheric_layer"], T, self.dt,
                                  self.state["total_precipitation"], in_place=True, level_axis=1, column=column)
        res = self._epi.out
        diags = [res["net_moistening_due_to_machine_learning"], res["column_heating_due_to_machine_learning"],
                 res["total_precipitation"]]
        self._part = bind_area_weighted_partials(diags, self.area)  # float64 diagnostics: the f64 reduction
        self._plan = LaunchPlan([self.bound, self._epi, self._part])  # one C-ABI call per step

    def step(self):
        """One step; returns the global [n_diag, 2] partials.  Without a process group this
        is the bound result buffer itself (valid until the next step: copy it to keep it)."""
        from . import _device
        from .distributed import combine_partials

        if self.bound is None:
            self._bind()
        h = _device.stream_handle()
        if self._in32 is not None:
            self._in32[0].copy_(self.state["air_temperature"])
            self._in32[1].copy_(self.state["specific_humidity"])
        self._plan(h)
        dist = torch.distributed
        if self.group is None and not (dist.is_available() and dist.is_initialized()):
            return self._part.result  # the bound result buffer, overwritten by the next step
        return combine_partials(self._part.result, self.group)


def make_stepper_workload(res: int = 96, seed: int = 0, device=None, group=None, precision: str = "f32"):
    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    shape = (6, NZ, res, res)
    base = torch.linspace(200.0, 1800.0, NZ, device=device, dtype=torch.float64)[None, :, None, None]
    state = {
        "air_temperature": 260.0 + 15.0 * torch.randn(shape, generator=g, device=device, dtype=torch.float64),
        "specific_humidity": 0.02 * torch.rand(shape, generator=g, device=device, dtype=torch.float64),
        "pressure_thickness_of_atmospheric_layer":
            base * (0.99 + 0.02 * torch.rand(shape, generator=g, device=device, dtype=torch.float64)),
        "total_precipitation": 1e-3 * torch.rand((6, res, res), generator=g, device=device, dtype=torch.float64),
    }
    area = 0.5 + 0.5 * torch.rand((6, res, res), generator=g, device=device, dtype=torch.float64)
    # the model's output normalisation fitted on tendencies of physical size (dQ1 ~ 1e-4 K/s,
    # dQ2 ~ 3e-8 kg/kg/s), so the state stays physical over many steps
    T, q = synthetic_state(8, seed, device, ntile=1)
    sample_T = T[0].reshape(NZ, -1).T.cpu().numpy()
    sample_q = q[0].reshape(NZ, -1).T.cpu().numpy()
    rng = np.random.default_rng(seed)
    sample_out = [rng.normal(0.0, 1e-4, sample_T.shape).astype(np.float32),
                  rng.normal(0.0, 3e-8, sample_T.shape).astype(np.float32)]
    model = DenseColumnModel.random(dense_2x256_config(), seed=1, sample_inputs=[sample_T, sample_q],
                                    sample_outputs=sample_out)
    return StepperWorkload(model, state, area, 900.0, 6 * res * res, group, precision=precision)


class _Result:
    """A fixed result buffer, read as ``.result`` like a bound launch's."""

    def __init__(self, result):
        self.result = result


@dataclasses.dataclass
class ShardedStepperWorkload:
    """BASELINE config #4 sharded as SURVEY.md 8(e) lays it out: this rank owns the rows
    [r0, r1) of the flattened (tile, y) rows of one global C<res> state, stored as a
    (z, rows, x) band, and per step runs the predict, the fused epilogue (in place) and
    the step's exchange: the global-mean partials of the 2-D diagnostics (net
    moistening, column heating, total precipitation), taken per grid row (6 doubles),
    all-gathered (RCCL on the GPU box) and folded in global row order, so the means have
    the same bits for any number of ranks; and the 3-D limiter profile (main.py:55-60),
    whose per-level counts are integers, summed on the rank and all-reduced (exact in
    float64 in any order: nz doubles per rank).  ``exchange_bytes``: this rank's bytes
    sent per step."""
    model: DenseColumnModel
    state: dict
    area: object
    dt: float
    rows: tuple
    ncol: int          # this rank's columns
    ncol_global: int
    group: object = None
    bound: object = None
    counts: object = None
    partials: object = None
    exchange_bytes: int = 0
    # > 1 without a process group: one rank's share of a ``stub_world``-rank run on one
    # GPU, the exchange stubbed by a local copy of the same bytes (this band's partials
    # replicated for every rank, then folded: the fold sees the full gathered row count)
    stub_world: int = 1
    _epi: object = None
    _lev: object = None
    _fold: object = None
    _diag: object = None
    _rep: object = None
    _res: object = None
    _plan: object = None

    def _bind(self):
        """Marshal every launch of the step once (predict, fused epilogue, row partials,
        limiter level counts; with the stubbed exchange also the fold into one result
        buffer): a step is then a handful of C-ABI calls on fixed buffers, no per-call
        Python marshalling (which, on one rank's 6,912 columns, took longer than the
        kernels).  The precipitation accumulates in place in the epilogue's column buffer."""
        from .distributed import bind_fold_rows_repeat, bind_step_partials
        from .stepper import BoundEpilogue

        T, q = self.state["air_temperature"], self.state["specific_humidity"]
        self.bound = self.model.bind([T, q], level_axes=[0, 0])
        dq1, dq2 = self.bound.outputs
        precip = self.state["total_precipitation"]
        column = torch.empty((7, precip.numel()), dtype=precip.dtype, device=precip.device)
        column[6].copy_(precip.reshape(-1))
        self.state["total_precipitation"] = column[6].view(precip.shape)
        self._epi = BoundEpilogue(dq1, dq2, q, self.state["pressure_thickness_of_atmospheric_layer"], T, self.dt,
                                  self.state["total_precipitation"], in_place=True, level_axis=0, column=column)
        res = self._epi.out
        nrows, nz = self.area.shape[0], q.shape[0]
        # [rows][3 (sum area*x, sum area) pairs]
        self.partials = torch.empty((nrows, 6), dtype=torch.float64, device=q.device)
        limiter = res["specific_humidity_limiter_active"]
        stub = self.stub_world > 1 and self.group is None
        if stub:
            self._rep = torch.empty((self.stub_world * nrows, 6), dtype=torch.float64, device=q.device)
            self._res = torch.empty(6 + nz, dtype=torch.float64, device=q.device)
            self._fold = bind_fold_rows_repeat(self.partials, self.stub_world, rep=self._rep, out=self._res[:6])
            level_out = self._res[6:]  # [nz] exact column counts
            self.exchange_bytes = 8 * (nrows * 6 + nz)
        else:
            level_out = torch.empty(nz, dtype=torch.float64, device=q.device)
        # the row partials and the limiter level counts in one launch (each with the bits
        # of its own: bind_area_row_partials / bind_level_sums)
        self._diag = bind_step_partials([res["net_moistening_due_to_machine_learning"],
                                         res["column_heating_due_to_machine_learning"],
                                         res["total_precipitation"]], self.area, limiter, out=self.partials,
                                        level_out=level_out)
        self._lev = _Result(level_out)
        # one C-ABI call per step: predict, epilogue, row partials + limiter counts (and,
        # with the stubbed exchange, this band's partials copied for every rank + the
        # fold, one launch)
        self._plan = LaunchPlan([self.bound, self._epi, self._diag])
        if self._fold is not None:
            self._plan.add(self._fold)

    def step(self):
        """One step; returns the 6 global partials followed by the nz limiter counts.  With
        the stubbed exchange this is the fold's result buffer itself (valid until the next
        step: copy it to keep it)."""
        from . import _device
        from .distributed import global_count_sums, global_row_sums, row_counts

        if self.bound is None:
            self._bind()
        self._plan(_device.stream_handle())
        limited = self._lev.result
        if self._fold is not None:  # stubbed exchange: the fold of every rank's (this band's) rows
            return self._res  # the result buffer, overwritten by the next step
        if self.counts is None:  # the bands are fixed: their sizes are exchanged once
            self.counts = row_counts(self.partials.shape[0], self.group)
            self.exchange_bytes = 8 * (max(self.counts) * 6 + limited.numel())
        means = global_row_sums(self.partials, self.group, self.counts)
        return torch.cat([means, global_count_sums(limited, self.group).to(means.device)])

    @staticmethod
    def means(total):
        """(global means of the three 2-D diagnostics, limiter global-sum profile)."""
        return total[0:6:2] / total[1:6:2], total[6:]


def make_sharded_stepper_workload(res: int = 96, rank: int = 0, world: int = 1, seed: int = 0, device=None,
                                  group=None, stub_exchange: bool = False):
    """Every rank generates the same global state (seeded) and keeps its row band.
    ``stub_exchange``: no process group, the exchange replaced by a local copy of the
    bytes ``world`` ranks would gather (one rank's share timed on one GPU)."""
    from .distributed import row_band

    wl = make_stepper_workload(res, seed=seed, device=device)
    r0, r1 = row_band(6 * res, rank, world)
    band3 = lambda a: a.permute(1, 0, 2, 3).reshape(NZ, 6 * res, res)[:, r0:r1].contiguous()  # noqa: E731
    band2 = lambda a: a.reshape(6 * res, res)[r0:r1].contiguous()  # noqa: E731
    state = {k: (band3(v) if v.dim() == 4 else band2(v)) for k, v in wl.state.items()}
    return ShardedStepperWorkload(wl.model, state, band2(wl.area), wl.dt, (r0, r1), (r1 - r0) * res,
                                  6 * res * res, group, stub_world=world if stub_exchange else 1)


@dataclasses.dataclass
class PredictMappmWorkload:
    """north_star's "fused predict + mappm at C384 x 79L": on this rank's band of the
    flattened (tile, y) rows of a C<res> state (z, rows, x), the config #2 predict of
    dQ1/dQ2 from T/q, then both tendencies remapped (mappm, kord 1, iv 1) from the state's
    edge pressures pe1 = 300 Pa + cumsum(delp) to 79 layers evenly spaced between the
    same top and surface (a per-column pressure-level regrid of the ML tendencies), all
    device-resident: one dense kernel and one two-field mappm kernel per step."""
    model: DenseColumnModel
    inputs: List
    outputs: List
    pe1: object
    pe2: object
    remapped: List
    ncol: int
    ncol_global: int
    flops_per_column: int
    bytes_per_column: int
    _bound: object = None
    _plans: object = None

    def step(self):
        from .mappm import MappmMultiPlan

        if self._bound is None:
            self._bound = self.model.bind(self.inputs, level_axes=[0, 0], outputs=self.outputs, out_level_axis=0)
            # both tendencies in one streaming pass over the shared edges
            self._plans = MappmMultiPlan(self.pe1, [o.view(o.shape[0], -1) for o in self.outputs], self.pe2, 1, 1,
                                         out=self.remapped)
        else:
            self._bound()
            self._plans()


def make_predict_mappm_workload(res: int = 384, rank: int = 0, world: int = 1, seed: int = 0, device=None,
                                precision: str = "f32"):
    from .distributed import row_band

    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    r0, r1 = row_band(6 * res, rank, world)
    band = lambda a: a.permute(1, 0, 2, 3).reshape(NZ, 6 * res, res)[:, r0:r1].contiguous()  # noqa: E731
    T, q = synthetic_state(res, seed, device)
    sample_T = T[0, :, :8, :8].reshape(NZ, -1).T.cpu().numpy()
    sample_q = q[0, :, :8, :8].reshape(NZ, -1).T.cpu().numpy()
    model = DenseColumnModel.random(dense_2x256_config(), seed=1, sample_inputs=[sample_T, sample_q])
    model.precision = precision
    T, q = band(T), band(q)
    ncol = (r1 - r0) * res
    g = torch.Generator(device=device)
    g.manual_seed(seed + 17)
    base = torch.linspace(200.0, 1800.0, NZ, device=device)[:, None]
    # the global state's delp (columns in flattened (tile, y, x) order), this rank's band
    # of rows: every rank count sees the same columns
    delp = base * (0.99 + 0.02 * torch.rand((NZ, 6 * res * res), generator=g, device=device))
    delp = delp[:, r0 * res:r1 * res].contiguous()
    top = torch.full((1, ncol), 300.0, device=device)
    pe1 = torch.cat([top, 300.0 + torch.cumsum(delp, 0)]).contiguous()
    frac = torch.linspace(0.0, 1.0, NZ + 1, device=device)[:, None]
    pe2 = (pe1[:1] + frac * (pe1[-1:] - pe1[:1])).contiguous()
    outs = [torch.empty_like(T), torch.empty_like(T)]
    remapped = [torch.empty((NZ, ncol), device=device), torch.empty((NZ, ncol), device=device)]
    cfg = model.config
    mappm_bytes = 4 * ((NZ + 1) + NZ + (NZ + 1) + NZ)
    return PredictMappmWorkload(model, [T, q], outs, pe1, pe2, remapped, ncol, 6 * res * res,
                                cfg.flops_per_column(), 4 * (cfg.k_in + cfg.k_out) + 2 * mappm_bytes)


@dataclasses.dataclass
class EmulatorWorkload:
    """BASELINE config #5 per GPU: the Zhao-Carr microphysics emulator on every column
    of a C384 79-level state (inputs in the Fortran [feature, sample] layout)."""
    emulator: object
    state: dict
    out: dict
    ncol: int
    flops_per_column: int
    bytes_per_column: int

    def step(self):
        return self.emulator(self.state, out=self.out)


def make_emulator_workload(res: int = 384, seed: int = 0, device=None, precision: str = "bf16x3",
                           rank: int = 0, world: int = 1):
    """``world`` > 1: this rank's band of the flattened (tile, y) rows only (config #5
    over ``world`` GPUs: 110,592 columns per GPU at C384 over 8)."""
    from .distributed import row_band
    from .emulator import MicrophysicsEmulator, zhao_carr_outputs

    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    r0, r1 = row_band(6 * res, rank, world)
    ncol = (r1 - r0) * res
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    lev = lambda a, b: torch.linspace(a, b, NZ, device=device)[:, None]
    T = lev(200.0, 300.0) + 5.0 * torch.randn((NZ, ncol), generator=g, device=device)
    q = 0.02 * torch.exp(-lev(0.0, 6.0)) * (0.2 + 0.8 * torch.rand((NZ, ncol), generator=g, device=device))
    qc = 1e-4 * torch.rand((NZ, ncol), generator=g, device=device) * (
        torch.rand((NZ, ncol), generator=g, device=device) < 0.3)
    delp = lev(200.0, 1800.0) * (0.98 + 0.04 * torch.rand((NZ, ncol), generator=g, device=device))
    state = {"air_temperature_input": T, "specific_humidity_input": q, "cloud_water_mixing_ratio_input": qc,
             "pressure_thickness_of_atmospheric_layer": delp,
             "air_temperature_after_last_gscond": T + 0.1 * torch.randn((NZ, ncol), generator=g, device=device),
             "specific_humidity_after_last_gscond": q * (0.95 + 0.1 * torch.rand((NZ, ncol), generator=g,
                                                                                 device=device))}
    sample = {k: v[:, :4096].T.contiguous().cpu().numpy() for k, v in state.items()}
    rng = np.random.default_rng(seed)
    sample_out = {}
    for o in zhao_carr_outputs(NZ):
        sc = 1e-3 if o.name == "total_precipitation" else (1e-5 if ("humid" in o.name or "cloud" in o.name) else 0.5)
        sample_out[o.name] = rng.normal(0, sc, (4096, o.nz)).astype(np.float32)
    emu = MicrophysicsEmulator.random(sample, sample_out, seed=seed, precision=precision)
    out = {(o.after or o.name): torch.empty((o.nz, ncol), device=device) for o in emu.outputs}
    cfg = emu.model.config
    return EmulatorWorkload(emu, state, out, ncol, cfg.flops_per_column(),
                            4 * (6 * NZ + cfg.k_out))

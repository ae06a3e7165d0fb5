"""A small labelled-array container with the slice of the xarray API that
fv3fit's Predictor boundary uses.

xarray is not installed in this image (nor on the GPU box), so the Predictor
classes accept either a real ``xarray.Dataset`` (duck-typed: ``ds[name].dims`` /
``.data`` / ``.coords``) or this ``Dataset``, and return the same kind.  The
semantics that matter for parity are xarray 0.19's (the reference pins
``xarray==0.19.0``, constraints.txt:315):

* ``Dataset.dims`` iterates in SORTED order (SortedKeysDict) — this is what makes
  fv3fit's ``stack`` order the sample dimensions alphabetically
  (external/fv3fit/fv3fit/_shared/stacking.py:12-27, test_stacking.py:86-94);
* iterating a Dataset yields its data-variable names in insertion order.

Data may be numpy arrays or torch tensors (CUDA tensors stay on device).
"""
import types
from collections import OrderedDict
from typing import Dict, Hashable, Iterable, Mapping, Optional, Sequence, Tuple

import numpy as np


def _shape(data) -> Tuple[int, ...]:
    shape = data.shape
    if type(shape) is tuple:  # numpy: already ints
        return shape
    return tuple(int(s) for s in shape)


def _to_numpy(data):
    if isinstance(data, np.ndarray):
        return data
    if hasattr(data, "detach"):  # torch
        return data.detach().cpu().numpy()
    return np.asarray(data)


class DataArray:
    def __init__(self, data, dims: Sequence[Hashable], coords: Optional[Mapping] = None,
                 attrs: Optional[Mapping] = None, name: Optional[Hashable] = None):
        if not hasattr(data, "shape"):
            data = np.asarray(data)
        dims = tuple(dims)
        if len(dims) != len(data.shape):
            raise ValueError(f"dims {dims} do not match data shape {tuple(data.shape)}")
        self.data = data
        self.dims = dims
        self.coords: Dict[Hashable, np.ndarray] = OrderedDict()
        for k, v in (coords or {}).items():
            if k in dims:
                self.coords[k] = np.asarray(v)
        self.attrs = dict(attrs or {})
        self.name = name

    @classmethod
    def _view(cls, data, dims, coords, attrs, name):
        """A DataArray over already-validated parts (a Dataset's own variable), no copies
        or checks: the hot path of ``Dataset.__getitem__``."""
        da = cls.__new__(cls)
        da.data, da.dims, da.coords, da.attrs, da.name = data, dims, coords, attrs, name
        return da

    @property
    def shape(self):
        return _shape(self.data)

    @property
    def sizes(self) -> Dict[Hashable, int]:
        return OrderedDict(zip(self.dims, self.shape))

    @property
    def values(self) -> np.ndarray:
        return _to_numpy(self.data)

    @property
    def dtype(self):
        return self.data.dtype

    def transpose(self, *dims) -> "DataArray":
        if len(dims) == 0:
            dims = tuple(reversed(self.dims))
        if set(dims) != set(self.dims):
            raise ValueError(f"transpose dims {dims} must be a permutation of {self.dims}")
        perm = [self.dims.index(d) for d in dims]
        data = self.data.permute(*perm) if hasattr(self.data, "permute") else np.transpose(self.data, perm)
        return DataArray(data, dims, self.coords, self.attrs, self.name)

    def __repr__(self):
        return f"<fv3net_amd.DataArray {self.name!r} dims={self.dims} shape={self.shape}>"


class Dataset:
    def __init__(self, data_vars: Optional[Mapping] = None, coords: Optional[Mapping] = None,
                 attrs: Optional[Mapping] = None):
        self._vars: "OrderedDict[Hashable, DataArray]" = OrderedDict()
        self._sizes: Dict[Hashable, int] = {}  # dim -> size over the variables (kept by __setitem__)
        self.coords: Dict[Hashable, np.ndarray] = OrderedDict((k, np.asarray(v)) for k, v in (coords or {}).items())
        self.attrs = dict(attrs or {})
        for k, v in (data_vars or {}).items():
            self[k] = v

    def __setitem__(self, name, value):
        if isinstance(value, tuple):
            value = DataArray(value[1], value[0])
        if not isinstance(value, DataArray):
            raise TypeError("Dataset values must be DataArray or (dims, data)")
        sizes = dict(zip(value.dims, value.shape))
        for d, n in sizes.items():
            other = self._sizes.get(d)
            if other is not None and other != n:
                raise ValueError(f"conflicting sizes for dimension {d!r}: {n} vs {other}")
        for k, v in value.coords.items():
            self.coords.setdefault(k, v)
        value.name = name
        replaced = name in self._vars
        self._vars[name] = value
        if replaced:  # the old variable's dims may be gone
            self._sizes = {}
            for v in self._vars.values():
                self._sizes.update(zip(v.dims, v.shape))
        else:
            self._sizes.update(sizes)

    def __getitem__(self, key):
        if isinstance(key, (list, tuple)) and not (isinstance(key, tuple) and key in self._vars):
            return Dataset({k: self[k] for k in key}, coords=self.coords, attrs=self.attrs)
        if key not in self._vars:
            if key in self.coords:  # a coordinate, as xarray's ds[name] gives it
                c = self.coords[key]
                return DataArray(c, (key,) if c.ndim == 1 else tuple(f"dim_{k}" for k in range(c.ndim)),
                                 {key: c} if c.ndim == 1 else None, name=key)
            raise KeyError(key)
        da = self._vars[key]
        coords = OrderedDict((d, self.coords[d]) for d in da.dims if d in self.coords)
        return DataArray._view(da.data, da.dims, coords, dict(da.attrs), key)

    def __contains__(self, key):
        return key in self._vars

    def __iter__(self):
        return iter(self._vars)

    def __len__(self):
        return len(self._vars)

    @property
    def data_vars(self):
        """Read-only view of the variables (assign through ``ds[name] = ...``, which keeps
        the dimension sizes and their conflict check in step)."""
        return types.MappingProxyType(self._vars)

    def keys(self):
        return self._vars.keys()

    @property
    def dims(self) -> Mapping[Hashable, int]:
        """Sorted mapping dim -> size (xarray 0.19 SortedKeysDict semantics)."""
        sizes = self._sizes
        return OrderedDict((d, sizes[d]) for d in sorted(sizes, key=str))

    @property
    def sizes(self):
        return self.dims

    def __repr__(self):
        return f"<fv3net_amd.Dataset vars={list(self._vars)} dims={dict(self.dims)}>"


# --- interop -----------------------------------------------------------------------
def is_xarray(obj) -> bool:
    mod = type(obj).__module__
    return mod.startswith("xarray")


def variable_dims(ds, name) -> Tuple[Hashable, ...]:
    return tuple(ds[name].dims)


def variable_data(ds, name):
    """The variable's data without forcing a host copy (torch stays torch)."""
    da = ds[name]
    data = getattr(da, "data", None)
    if data is None:
        data = da.values
    return data


def infer_dimension_order(ds) -> Tuple[Hashable, ...]:
    """First-seen dim order across variables (stacking.py:30-37)."""
    order = []
    for name in ds:
        for d in ds[name].dims:
            if d not in order:
                order.append(d)
    return tuple(order)


def dataset_dims(ds) -> Iterable[Hashable]:
    """Dimension names in the order fv3fit's stack() iterates them: sorted
    (xarray 0.19).  For a real xarray object we sort too, which is what 0.19 did."""
    return sorted(ds.dims, key=str)

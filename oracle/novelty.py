"""TEST INFRASTRUCTURE ONLY — the checker of csrc/novelty.hip, never the product path.

numpy restatement of the out-of-sample composite's arithmetic, in the reference's dtype
flow (reference files under /root/reference/external/fv3fit/fv3fit):
* MinMaxNoveltyDetector.predict      sklearn/_min_max_novelty_detector.py:86-115 (pack:
  _shared/packer.py:106-127 (clip, variables' features in order; to_stacked_array's
  promoted dtype); MinMaxScaler.transform (scikit-learn): X *= scale_; X += min_ in place)
* taper_mask / taper_ramp / taper_decay   _shared/taper_function.py:6-35
* OutOfSampleModel.predict's products     _shared/models.py:392-398
Pinned by tests/test_novelty.py: the taper functions against the reference's own KATs
(external/fv3fit/tests/test_taper.py:19-60), the scaler against scikit-learn's
MinMaxScaler (importable here) fitted and applied on the same data.
"""
import numpy as np


def pack(features):
    """[ncol, nfeat_v] arrays of the variables, in order -> [ncol, nfeat] (numpy's promotion)."""
    return np.concatenate([np.asarray(f) for f in features], axis=1)


def minmax_scores(X, scale, min_):
    """score per row of the packed features X (MinMaxScaler.transform in place, in X's dtype)."""
    X = np.array(X, copy=True)
    X *= scale
    X += min_
    scores_larger_than_max = np.maximum(X.max(axis=1) - 1, 0)
    scores_smaller_than_min = np.maximum(-1 * X.min(axis=1), 0)
    return scores_larger_than_max + scores_smaller_than_min


def taper_mask(novelty_score, cutoff=0, **kwargs):
    return np.where(np.asarray(novelty_score) > cutoff, 0, 1)


def taper_ramp(novelty_score, ramp_min=0, ramp_max=1, **kwargs):
    unclipped = (ramp_max - np.asarray(novelty_score)) / (ramp_max - ramp_min)
    return np.clip(unclipped, 0, 1)


def taper_decay(novelty_score, threshold=0, rate=0.5, **kwargs):
    return np.minimum(rate ** (np.asarray(novelty_score) - threshold), 1)


TAPERS = {"taper_mask": taper_mask, "taper_ramp": taper_ramp, "taper_decay": taper_decay}

"""Convert a reference MinMaxNoveltyDetector directory (fv3fit/sklearn/
_min_max_novelty_detector.py:135-160: ``minmax.pkl`` (joblib pickle of the fitted
scikit-learn MinMaxScaler) + ``metadata.bin``) into this build's format: ``minmax.npz``
(the scaler's arrays) + the same ``metadata.bin`` + the name file ``minmax``.

    python tools/export_minmax.py <reference model dir> <output dir>

It UNPICKLES the reference's file: run it only where that model file is trusted and
joblib / scikit-learn are installed (the maintainer's training environment).  The
library itself never loads pickles (fv3net_amd/novelty.py).
"""
import os
import shutil
import sys

import numpy as np


def main(src: str, dst: str) -> None:
    import joblib  # the reference's own serializer

    with open(os.path.join(src, "minmax.pkl"), "rb") as f:
        scaler = joblib.load(f)["scaler"]
    os.makedirs(dst, exist_ok=True)
    np.savez(os.path.join(dst, "minmax.npz"), scale_=scaler.scale_, min_=scaler.min_,
             data_min_=scaler.data_min_, data_max_=scaler.data_max_)
    shutil.copy(os.path.join(src, "metadata.bin"), os.path.join(dst, "metadata.bin"))
    with open(os.path.join(dst, "name"), "w") as f:
        print("minmax", file=f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

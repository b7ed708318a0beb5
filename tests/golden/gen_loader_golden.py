"""tests/golden/loader.npz: the REFERENCE's KalmanNet/data_loader.py:load_vehicle_dataset run on small
CSVs written by trajectory_generation_amd.dataset.frames from deterministic synthetic histories
(tests/test_dataset.py rebuilds the same CSVs).  Build container only:  python tests/golden/gen_loader_golden.py"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def synthetic_histories():
    rng = np.random.default_rng(11)
    B, T = 10, 30
    return rng.normal(size=(B, T + 1, 6)), rng.normal(size=(B, T, 2)), 0.01


def main():
    from trajectory_generation_amd.dataset import frames
    sys.path.insert(0, "/root/reference/KalmanNet")
    import data_loader as DL
    X, U, Ts = synthetic_histories()
    with tempfile.TemporaryDirectory() as d:
        clean, noisy = frames(X, U, np.arange(X.shape[0]), Ts)
        clean.to_csv(os.path.join(d, "c.csv"), index=False)
        noisy.to_csv(os.path.join(d, "n.csv"), index=False)
        tr, va, te = DL.load_vehicle_dataset(os.path.join(d, "n.csv"), os.path.join(d, "c.csv"), T_steps=25)
    arrs = {}
    for name, part in (("train", tr), ("val", va), ("test", te)):
        for k, t in zip("yux", part):
            arrs[f"{name}_{k}"] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "loader.npz"), **arrs)
    print({k: v.shape for k, v in arrs.items()})


if __name__ == "__main__":
    main()

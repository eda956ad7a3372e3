"""Copies the labelled cone crops of the reference's plain-CSV data file
(cones_clouds/cones.csv: one row per crop, x / y / z / intensity as JSON lists, color 1..3)
into tests/golden/cones_csv.npz: points (P, 4) float32 in crop order, offsets (C + 1), labels
(C). The CSV holds 2 crops; the reference's other crops are in cones_clouds/cones.pkl, a pickle,
which is not loaded (serialized files are read only by loaders that execute nothing).
    python tests/golden/make_cones_csv.py [/root/reference/cones_clouds/cones.csv]"""
import csv
import json
import os
import sys

import numpy as np

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/cones_clouds/cones.csv"
rows = list(csv.DictReader(open(src)))
pts, offs, labels = [], [0], []
for r in rows:
    cols = [np.asarray(json.loads(r[k]), np.float64) for k in ("x", "y", "z", "intensity")]
    n = len(cols[0])
    assert all(len(c) == n for c in cols)
    pts.append(np.stack(cols, 1).astype(np.float32))
    offs.append(offs[-1] + n)
    labels.append(int(r["color"]))
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cones_csv.npz")
np.savez(out, points=np.concatenate(pts), offsets=np.asarray(offs, np.int64), labels=np.asarray(labels, np.int64))
print(out, len(labels), "crops", offs[-1], "points")

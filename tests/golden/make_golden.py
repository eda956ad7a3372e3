#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz: inputs and CPU-restatement outputs of the hot path.

The reference has no golden data of its own and cannot run here, so these
fixtures are produced by the oracle (oracle/cg_oracle.cpp, PCL's std::sort voxel order) and cross-checked at generation time
against the independent numpy restatement (tests/np_reference.py). They pin both restatements
(and the host libm they call) and give the GPU tests size-bounded vectors that need no
generator. Cases: two C1 frames (16 rings x 1024 columns, simulation params) and every
known-answer cloud of tests/kat_clouds.py.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import cones_perception_amd as cp  # noqa: E402
import kat_clouds as KC  # noqa: E402
import np_reference as R  # noqa: E402
import oracle_py as O  # noqa: E402


def outputs(params, msg, mode):
    if mode == O.MODE_GROUND:
        g, hdr = O.run(params, msg, mode)
        return {"hdr": hdr, "ground": g}
    det, hdr = O.run(params, msg, mode)
    return {"hdr": hdr, "voxels": det.voxels, "labels": det.labels, "offsets": det.cluster_offsets,
            "indices": det.cluster_indices, "centroids": det.centroids}


def save_case(name, pts_raw, point_step, over):
    params = cp.load_params("simulation", over)
    n = pts_raw.size // point_step
    msg = cp.frame_cloud(pts_raw, point_step) if n else cp.PointCloud2.from_xyzi(np.zeros((0, 4), np.float32))
    arrays = {"input": pts_raw, "point_step": np.array(point_step), "params": np.array(json.dumps(over))}
    for mode, tag in ((O.MODE_PIPELINE, "pipeline"), (O.MODE_DETECT, "detect"), (O.MODE_GROUND, "ground")):
        for k, v in outputs(params, msg, mode).items():
            arrays[f"{tag}_{k}"] = v
    # cross-check against the numpy restatement before saving (it sums each voxel in point
    # order: compared with the oracle's ORDER_STABLE; the fixtures hold PCL's order)
    prm = {**cp.GROUND_PARAMS, **cp.PROFILES["simulation"], **over}
    ref = R.pipeline(msg.xyzi(), prm, ground=True)
    st, _ = O.run(params, msg, O.MODE_PIPELINE, O.ORDER_STABLE)
    assert int(arrays["pipeline_hdr"][2]) == ref["M"], name
    assert np.array_equal(st.voxels.view(np.uint32), ref["vox"].view(np.uint32)) or \
        np.isnan(ref["vox"]).any(), name
    assert [list(c) for c in st.clusters] == ref["clusters"] or len(ref["clusters"]) > 16, name
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    print(f"{name}: N={n} K={int(arrays['pipeline_hdr'][1])} M={int(arrays['pipeline_hdr'][2])} "
          f"V={int(arrays['pipeline_hdr'][3])} C={int(arrays['pipeline_hdr'][4])}")


def main():
    raw = cp.synth_frames(2, first_frame=0, rings=16, cols=1024)
    for f in range(2):
        save_case(f"c1_frame{f}", raw[f].copy(), 16, {})
    for name, pts, over, _ in KC.all_kats():
        msg = cp.PointCloud2.from_xyzi(pts)
        save_case(f"kat_{name}", np.ascontiguousarray(msg.data), 16, over)


if __name__ == "__main__":
    main()

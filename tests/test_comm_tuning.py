"""tools/comm_bench.py --recommend: the settings derived from a sweep's measurements (CPU; the 8-GPU sweep
itself runs where 8 GPUs are), and bench.py's adoption rule for them."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import comm_bench  # noqa: E402


def _rows(world=8):
    rows = []
    for env, scale in (({}, 1.0), ({"NCCL_MIN_NCHANNELS": "16"}, 0.9), ({"NCCL_ALGO": "Tree"}, 1.2)):
        for b, us in ((77312, 10.0), (454720, 14.0), (4194304, 40.0), (26214400, 150.0)):
            rows.append({"impl": "rccl", "world": world, "dtype": "fp32", "bytes": b, "us_per_op": us * scale,
                         "correct": True, "rccl_env": env})
            small = {77312: 5.0, 454720: 11.0, 4194304: 60.0}.get(b)
            if small is not None:
                rows.append({"impl": "rccl+xgmi_small", "world": world, "dtype": "fp32", "bytes": b,
                             "us_per_op": small, "correct": True, "rccl_env": env})
    return rows


def test_recommend_picks_fastest_variant_and_crossover():
    rec = comm_bench.recommend(_rows(), 8)
    assert rec["world"] == 8
    assert rec["env"]["NCCL_MIN_NCHANNELS"] == "16"
    # the one-shot kernel wins up to 455 KB (5 < 9, 11 < 12.6) and loses at 4 MB (60 > 36)
    assert rec["env"]["RINGDP_P2P_ALLREDUCE_MAX_BYTES"] == "454720"


def test_recommend_ignores_wrong_results_and_other_worlds():
    rows = _rows()
    for r in rows:
        if r["impl"] == "rccl+xgmi_small" and r["bytes"] == 77312:
            r["correct"] = False  # a failed check never becomes a recommendation
    rows += [dict(r, world=4, us_per_op=0.1) for r in _rows(4)]
    rec = comm_bench.recommend(rows, 8)
    assert rec["env"]["RINGDP_P2P_ALLREDUCE_MAX_BYTES"] == "0"
    assert json.loads(rec["evidence"]["chosen_variant"]) == {"NCCL_MIN_NCHANNELS": "16"}

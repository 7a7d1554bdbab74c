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


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("ringdp_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_recommend_records_identity():
    rows = _rows()
    for r in rows:
        r["identity"] = {"arch": "gfx950", "host": "node1", "rccl": "2.26.6"}
    assert comm_bench.recommend(rows, 8)["identity"] == {"arch": "gfx950", "host": "node1", "rccl": "2.26.6"}
    rows[0]["identity"] = {"arch": "gfx942", "host": "node1", "rccl": "2.26.6"}  # mixed sweep: adopt nowhere
    assert comm_bench.recommend(rows, 8)["identity"] is None


def test_bench_adopts_tuning_only_where_measured(tmp_path, monkeypatch):
    """comm_tuning.json changes NCCL_* / RINGDP_* settings only at the world size, device type,
    host and RCCL version it was measured on; anything else is reported and ignored."""
    bench = _bench()
    here = {"arch": "gfx950", "host": "node1", "rccl": "2.26.6"}
    path = tmp_path / "comm_tuning.json"
    rec = {"world": 8, "env": {"RINGDP_TEST_TUNING_KNOB": "454720"}, "identity": dict(here)}
    path.write_text(json.dumps(rec))
    monkeypatch.delenv("RINGDP_TEST_TUNING_KNOB", raising=False)
    r = bench._adopt_comm_tuning(str(path), 4, here)
    assert not r["adopted"] and "world" in r["reason"] and "RINGDP_TEST_TUNING_KNOB" not in os.environ
    r = bench._adopt_comm_tuning(str(path), 8, dict(here, host="other"))
    assert not r["adopted"] and "host" in r["reason"] and "RINGDP_TEST_TUNING_KNOB" not in os.environ
    path.write_text(json.dumps(dict(rec, identity=None)))  # a file without identity is never adopted
    assert not bench._adopt_comm_tuning(str(path), 8, here)["adopted"]
    path.write_text(json.dumps(rec))
    r = bench._adopt_comm_tuning(str(path), 8, here)
    assert r["adopted"] and os.environ["RINGDP_TEST_TUNING_KNOB"] == "454720"
    monkeypatch.setenv("RINGDP_TEST_TUNING_KNOB", "7")  # the environment wins over the file
    assert bench._adopt_comm_tuning(str(path), 8, here)["env"]["RINGDP_TEST_TUNING_KNOB"] == "7"


def test_comm_model_placement_and_scaling():
    """ringdp.utils.comm_model: the constants reproduce the measured shared-GPU floors, the ConvNet's N=8
    placement follows (369 KB bucket split off, the 76 KB last bucket inline) and the scaling model reports
    exposed time / efficiency with and without the one-shot path."""
    from ringdp.utils import comm_model as cm

    assert abs(cm.est_us(77312, 2) - 8.55) < 1.0 and abs(cm.est_us(77312, 4) - 15.1) < 1.5
    assert cm.est_us(369_000, 8) > cm.SPLIT_MIN_US > cm.est_us(76_000, 1)
    plan = [{"bytes": 369_000, "placement": "inline"}, {"bytes": 76_000, "placement": "inline (last)"}]
    m = cm.scaling_model(plan, 3400.0, 1)  # the one-rank run captured both inline; at N=8 bucket 0 splits
    assert m["8"]["placement"] == ["split", "inline (last)"] and m["2"]["placement"] == ["inline", "inline (last)"]
    assert m["8"]["exposed_us_ring"] == round(cm.est_us(76_000, 8), 2)
    assert m["8"]["E_ring"] > 0.98
    one = cm.scaling_model([{"bytes": 454_720, "placement": "inline (last)"}], 80.0, 1)
    assert one["8"]["E_oneshot"] > one["8"]["E_ring"] and one["8"]["E_ring"] < 0.8

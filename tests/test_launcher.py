"""``python -m ringdp.run`` / ``python -m ringdp.launch``: worker env contract,
legacy ``--local-rank`` argv, failure propagation, --max-restarts, and a two-launcher "multi-node"
rendezvous on one host (gloo / host ring)."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _script(tmp_path, body):
    p = tmp_path / "worker.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def _launch(args, timeout=120, env=None):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.pop("OMP_NUM_THREADS", None)
    if env:
        e.update(env)
    return subprocess.run([sys.executable, "-m"] + args, cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=timeout)


ENV_DUMP = """
import json, os, sys
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
        "MASTER_PORT", "TORCHELASTIC_RESTART_COUNT", "OMP_NUM_THREADS"]
out = {k: os.environ.get(k) for k in keys}
out["argv"] = sys.argv[1:]
out_dir = [a for a in sys.argv[1:] if not a.startswith("--local")][0]
with open(os.path.join(out_dir, f"env_{os.environ['RANK']}.json"), "w") as f:
    json.dump(out, f)
"""


def test_run_env_contract(tmp_path):
    script = _script(tmp_path, ENV_DUMP)
    port = _port()
    r = _launch(["ringdp.run", "--nproc-per-node", "3", "--master-port", str(port), script, str(tmp_path)])
    assert r.returncode == 0, r.stderr
    envs = [json.load(open(tmp_path / f"env_{i}.json")) for i in range(3)]
    for i, e in enumerate(envs):
        assert e["RANK"] == str(i) and e["LOCAL_RANK"] == str(i)
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3" and e["GROUP_RANK"] == "0"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == str(port)
        assert e["TORCHELASTIC_RESTART_COUNT"] == "0"
        assert e["OMP_NUM_THREADS"] == "1"
        assert e["argv"] == [str(tmp_path)]  # torchrun style: no --local-rank


def test_legacy_launch_passes_local_rank(tmp_path):
    script = _script(tmp_path, ENV_DUMP)
    r = _launch(["ringdp.launch", "--nproc_per_node", "2", "--master_port", str(_port()), script, str(tmp_path)])
    assert r.returncode == 0, r.stderr
    for i in range(2):
        e = json.load(open(tmp_path / f"env_{i}.json"))
        assert e["argv"] == [f"--local-rank={i}", str(tmp_path)]  # torch.distributed.launch order
    r = _launch(["ringdp.launch", "--use-env", "--nproc_per_node", "2", "--master_port", str(_port()), script,
                 str(tmp_path)])
    assert r.returncode == 0, r.stderr
    assert json.load(open(tmp_path / "env_1.json"))["argv"] == [str(tmp_path)]


def test_failure_propagates_and_peers_are_stopped(tmp_path):
    script = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # must be terminated by the launcher
    """)
    t0 = time.time()
    r = _launch(["ringdp.run", "--nproc-per-node", "2", "--master-port", str(_port()), "--grace-period", "2",
                 script], timeout=90)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert time.time() - t0 < 60


def test_max_restarts(tmp_path):
    script = _script(tmp_path, """
        import os, sys
        if os.environ["TORCHELASTIC_RESTART_COUNT"] == "0" and os.environ["RANK"] == "0":
            sys.exit(1)
        open(os.path.join(sys.argv[1], "ok_" + os.environ["RANK"] + "_" + os.environ["TORCHELASTIC_RESTART_COUNT"]), "w").close()
    """)
    r = _launch(["ringdp.run", "--nproc-per-node", "2", "--master-port", str(_port()), "--max-restarts", "1",
                 "--grace-period", "2", script, str(tmp_path)])
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "ok_0_1").exists() and (tmp_path / "ok_1_1").exists()
    r = _launch(["ringdp.run", "--nproc-per-node", "2", "--master-port", str(_port()), "--max-restarts", "0",
                 "--grace-period", "2", script, str(tmp_path)])
    assert r.returncode != 0


def test_two_launchers_simulate_two_nodes(tmp_path):
    """--nnodes 2 --node-rank {0,1} on one host: 4 ranks rendezvous and all-reduce over the host ring."""
    script = _script(tmp_path, """
        import os, sys, torch
        import ringdp.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(dist.get_rank() + 1)])
        dist.all_reduce(t)
        with open(os.path.join(sys.argv[1], "sum_" + os.environ["RANK"]), "w") as f:
            f.write(f"{dist.get_world_size()} {int(t.item())} {os.environ['LOCAL_RANK']} {os.environ['GROUP_RANK']}")
        dist.destroy_process_group()
    """)
    port = _port()
    e = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = [subprocess.Popen([sys.executable, "-m", "ringdp.run", "--nnodes", "2", "--node-rank", str(n),
                               "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", str(port),
                               script, str(tmp_path)], cwd=ROOT, env=e, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for n in (0, 1)]
    for p in procs:
        _, err = p.communicate(timeout=180)
        assert p.returncode == 0, err
    for r in range(4):
        ws, total, lr, gr = (tmp_path / f"sum_{r}").read_text().split()
        assert ws == "4" and total == "10" and lr == str(r % 2) and gr == str(r // 2)

"""The reference-recipe examples (W1 / W2, spawn and launch entrypoints) run end to end on the
host-ring backend (BASELINE config #1: ConvNet DDP world_size=2 on CPU via spawn)."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, env=None, timeout=300):
    e = dict(os.environ, PYTHONPATH=ROOT)
    if env:
        e.update(env)
    r = subprocess.run([sys.executable] + cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_mnist_mpspawn_cpu():
    out = _run(["examples/mnist_mpspawn.py", "-g", "2", "--cpu", "--epochs", "1", "--max-steps", "3",
                "--log-every", "1"], env={"MASTER_PORT": str(_port())})
    assert "Epoch [1/1], Step [3/300], Loss:" in out and "Training complete in:" in out


def test_mnist_launch_cpu():
    out = _run(["-m", "ringdp.launch", "--nproc_per_node=2", f"--master_port={_port()}", "examples/mnist_launch.py",
                "--cpu", "--epochs", "1", "--max-steps", "2", "--log-every", "1"])
    assert "Step [2/300]" in out


def test_cifar_resnet_mp_cpu():
    out = _run(["examples/cifar_resnet_mp.py", "--ngpus_per_node", "2", "--cpu", "--epochs", "1", "--max-steps", "2",
                "--batch-size", "8", "--workers", "2", "--dist-url", f"tcp://127.0.0.1:{_port()}"])
    assert "== step: [  2/" in out and "Training Finished" in out


def test_cifar_resnet_launch_cpu():
    out = _run(["-m", "ringdp.run", "--nproc-per-node=2", f"--master-port={_port()}", "examples/cifar_resnet_launch.py",
                "--cpu", "--epochs", "1", "--max-steps", "2", "--batch-size", "8", "--workers", "2"])
    assert "Training Finished" in out

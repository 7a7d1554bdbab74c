"""Write a profiles/ evidence summary from a tools/profile_all.sh run in gpurun_out/.

python tools/make_summary.py profiles/NAME.md "title" "free-text notes"
"""
import contextlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_summary  # noqa: E402

BENCHES = [("bench_convnet", "ConvNet (default `python bench.py`, hipGraph)"),
           ("bench_convnet_b100", "ConvNet, reference batch 100/rank"),
           ("bench_resnet18", "ResNet-18 CIFAR-shape B=256"),
           ("bench_resnet50", "ResNet-50 ImageNet-shape B=256"),
           ("bench_vit", "ViT-B/16 B=128 bf16"),
           ("bench_vit_fp8", "ViT-B/16 B=128 fp8 linears")]


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def json_lines(path):
    return [line for line in open(path).read().splitlines() if line.startswith("{")]


def kernel_table(model, n=14):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        prof_summary.main(f"gpurun_out/prof_{model}/run_kernel_stats.csv", n)
    return buf.getvalue()


def main(out, title, notes):
    rows = []
    for name, label in BENCHES:
        d = last_json(f"gpurun_out/{name}.log")
        if d:
            rows.append(f"| {label} | {d['config']['per_rank_batch']} | {d['value']:,.0f} | {d['ms_per_step']} | "
                        f"{d['dtype'].split(' (')[0]} | {d['config']['hipgraph']} |")
    tests = open("gpurun_out/pytest_gpu.log").read().strip().splitlines()[-1]
    parts = [
        f"# {title}\n",
        f"Collected with `tools/profile_all.sh` in one gpurun call on 1x MI355X (gfx950). {notes}\n",
        "## GPU tests\n", "```", tests, "```\n",
        "## bench.py (1 GPU; the round-end driver measures 2/4/8)\n",
        "| config | per-rank batch | images/s | ms/step | dtype | hipGraph |",
        "|---|---:|---:|---:|---|---|", *rows, "",
        "## ConvNet step kernels (default batch, eager, rocprofv3 --kernel-trace --stats)\n", kernel_table("convnet"),
        "## ResNet-50 step kernels (B=256)\n", kernel_table("resnet50"),
        "## ViT-B/16 step kernels (B=128, bf16)\n", kernel_table("vit"),
        "## ConvNet per-kernel microbenchmark (tools/kbench.py, HIP-event medians)\n",
        "```", *json_lines("gpurun_out/kbench.log"), "```\n",
        "## GEMM core microbenchmark (tools/gemm_bench.py; conv rows: [us, TFLOP/s])\n",
        "```", *json_lines("gpurun_out/gemm_bench.log"), "```",
    ]
    with open(out, "w") as f:
        f.write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:4])

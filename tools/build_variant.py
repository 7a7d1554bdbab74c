"""Build an A/B variant of the extension: one .hip source recompiled with extra -D flags, linked
with the current in-tree objects into variants/<name>.so (run with RINGDP_EXT_PATH=variants/<name>.so,
tools/gpu_ab_variants.sh).  usage: python tools/build_variant.py NAME csrc/kernels/x.hip -DFOO=1 ..."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("ringdp_build", ROOT / "ringdp" / "_build.py")
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)

name, src, defs = sys.argv[1], (ROOT / sys.argv[2]).resolve(), sys.argv[3:]
b.build(verbose=False)
out_dir = ROOT / __import__("os").environ.get("RINGDP_VARIANT_DIR", "variants")
out_dir.mkdir(exist_ok=True)
obj = out_dir / f"{name}.{src.stem}.o"
cmd = b._compile_cmd(src, obj)
cmd = cmd[:-4] + defs + cmd[-4:]
b._run(cmd)
hip, cpp = b._sources()
objs = [obj if s == src else b._obj_for(s) for s in hip + cpp]
b._run(b._link_cmd(objs, out_dir / f"{name}.so"))
print(out_dir / f"{name}.so")

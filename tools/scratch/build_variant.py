"""Link a variant of the extension with extra -D flags on ONE .hip file (A/B experiments).

usage: python tools/build_variant.py <out.so> <kernels/file.hip> -DFOO -DBAR=2
The other objects come from the normal in-tree build (run ``python __graft_entry__.py build`` first).
On the GPU box: copy the variant over ringdp/_C*.so before importing ringdp."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("_b", ROOT / "ringdp" / "_build.py")
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)

out, src, flags = Path(sys.argv[1]), b.CSRC / sys.argv[2], sys.argv[3:]
hip, cpp = b._sources()
objs = []
for s in hip + cpp:
    if s == src:
        o = Path("/tmp") / (out.stem + "_" + s.stem + ".o")
        cmd = b._compile_cmd(s, o)
        b._run(cmd[:1] + flags + cmd[1:])
        objs.append(o)
    else:
        objs.append(b._obj_for(s))
out.parent.mkdir(parents=True, exist_ok=True)
b._run(b._link_cmd(objs, out))
print("built", out)

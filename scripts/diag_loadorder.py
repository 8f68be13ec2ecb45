"""Diagnostic: does the engine work whichever HIP runtime copy is loaded
first (system ROCm via the .so, or torch's bundled one)?"""
import subprocess
import sys

SNIPS = {
    "lib_only": "import hdfs_native_ec as H",
    "lib_then_torch": "import hdfs_native_ec as H; import torch; print('cuda', torch.cuda.is_available())",
    "torch_then_lib": "import torch; print('cuda', torch.cuda.is_available()); import hdfs_native_ec as H",
}
BODY = """
import sys, numpy as np
c = H.Coder(6, 3, 0)
d = [bytes([i]*4096) for i in range(6)]
p = c.encode(d)
print('encode ok', [x[:4] for x in p])
"""
for name, pre in SNIPS.items():
    code = "import sys; sys.path.insert(0,'hdfs-native_amd'); " + pre + "\n" + BODY
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    print(f"== {name}: rc={r.returncode}\n{r.stdout}{r.stderr[-2000:]}", flush=True)

"""Per-kernel register / spill / LDS usage of kernels.hip from hipcc's resource-usage remarks,
for two trees side by side (e.g. HEAD against the working tree):

    python scripts/resource_usage.py            # HEAD vs working tree, kernels that changed
    python scripts/resource_usage.py --all      # every kernel

No GPU needed (device-only compile for gfx950)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ['TotalSGPRs', 'VGPRs', 'SGPRs Spill', 'VGPRs Spill', 'ScratchSize [bytes/lane]',
        'Occupancy [waves/SIMD]', 'LDS Size [bytes/block]']


def usage(csrc, inc):
    out = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17',
                          '-mllvm', '-amdgpu-atomic-optimizer-strategy=None', '-I', inc, '-c',
                          os.path.join(csrc, 'kernels.hip'), '-o', os.devnull, '--cuda-device-only',
                          '-Rpass-analysis=kernel-resource-usage'],
                         capture_output=True, text=True).stderr
    d, cur = {}, None
    for line in out.splitlines():
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            cur = re.sub(r'^_ZN12_GLOBAL__N_1\d+', '', m.group(1))[:48]
            d[cur] = {}
            continue
        m = re.search(r'remark:\s+([A-Za-z \[\]/]+): (\d+)', line)
        if cur and m:
            d[cur][m.group(1).strip()] = int(m.group(2))
    return d


def main():
    with tempfile.TemporaryDirectory() as t:
        old = os.path.join(t, 'csrc')
        os.makedirs(old)
        for f in os.listdir(os.path.join(ROOT, 'replicat_amd', 'csrc')):
            blob = subprocess.run(['git', 'show', f'HEAD:replicat_amd/csrc/{f}'], cwd=ROOT,
                                  capture_output=True).stdout
            with open(os.path.join(old, f), 'wb') as fh:
                fh.write(blob)
        inc = os.path.join(ROOT, 'include')
        a, b = usage(old, inc), usage(os.path.join(ROOT, 'replicat_amd', 'csrc'), inc)
    for k in sorted(b):
        diff = [(x, a.get(k, {}).get(x), b[k].get(x)) for x in KEYS if a.get(k, {}).get(x) != b[k].get(x)]
        if diff or '--all' in sys.argv:
            print(k, diff or [(x, b[k].get(x)) for x in KEYS])


if __name__ == '__main__':
    main()

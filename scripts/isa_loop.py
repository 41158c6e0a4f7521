"""Instruction mix of a kernel's large basic blocks from the gfx950 ISA (no GPU needed):

    python scripts/isa_loop.py [kernel-substring] [--dump BLOCK]

Compiles kernels.hip with the library's flags to assembly (cached in /tmp) and prints, for each
basic block of more than 200 instructions of the matching kernels, the instruction count, the
VALU count and the most frequent opcodes -- the tile kernel's loop body is the largest block."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def isa(src=os.path.join(ROOT, 'replicat_amd', 'csrc', 'kernels.hip'), extra=()):
    out = '/tmp/rc_kernels_isa.s'
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-mllvm',
                    '-amdgpu-atomic-optimizer-strategy=None', '-I', os.path.join(ROOT, 'include'),
                    *extra, '-S', '--cuda-device-only', src, '-o', out], check=True,
                   stderr=subprocess.DEVNULL)
    return open(out).read().split('\n')


def blocks(lines, kernel):
    res = {}
    for i, l in enumerate(lines):
        m = re.match(r'^(_ZN\S*' + re.escape(kernel) + r'\S*):', l)
        if not m:
            continue
        end = next(k for k in range(i, len(lines)) if lines[k].startswith('.Lfunc_end'))
        cur = None
        out = []
        for ln in lines[i:end]:
            if re.match(r'^(\.LBB\d+_\d+|_ZN\S+):', ln):
                cur = [ln.split(':')[0], []]
                out.append(cur)
            elif cur and ln.startswith('\t') and not ln.strip().startswith((';', '.')):
                cur[1].append(ln.strip())
        res[m.group(1)] = out
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    kernel = args[0] if args else 'rc_tile_kernel'
    dump = sys.argv[sys.argv.index('--dump') + 1] if '--dump' in sys.argv else None
    defs = [a for a in sys.argv[1:] if a.startswith('-D')]
    for fn, bl in blocks(isa(extra=defs), kernel).items():
        print(fn[:90])
        for name, ins in bl:
            if dump and name == dump:
                print('\n'.join(ins))
            if len(ins) < 200:
                continue
            c = collections.Counter(i.split()[0] for i in ins)
            valu = sum(v for k, v in c.items() if k.startswith('v_'))
            print(f'  {name}: {len(ins)} instructions, {valu} VALU')
            print('   ', ', '.join(f'{k} {v}' for k, v in c.most_common(24)))


if __name__ == '__main__':
    main()

"""The bench lines of a final validation log (scripts/gpu_final.sh: '== args' then the line), one
row each: value, ms/step, tile kernel, frac / frac_read, profile_frac, chain, traffic / bytes
read, parity, pipelined steps, in-sequence ms/step, read probe, host path, CPU baseline, warm-up.

    python scripts/final_table.py gpurun_out/final6/configs.log
"""
import json
import sys


def rows(path):
    args = None
    for line in open(path):
        if line.startswith('== '):
            args = line[3:].strip()
        elif line.startswith('{'):
            yield args, json.loads(line)


def main():
    for args, d in rows(sys.argv[1]):
        r = d['roofline']
        tr = r.get('traffic')
        out = {'args': args, 'value': d['value'], 'ms_per_step': d['ms_per_step'],
               'tile_ms': r['kernel_ms'], 'frac': r.get('frac'), 'frac_read': r.get('frac_read'),
               'profile_frac': r.get('profile_frac'), 'chain_ms': r['chain_kernel_ms'],
               'traffic_over_read': round(tr / r['bytes_read'], 4) if tr and r.get('bytes_read') else None,
               'parity': d['parity_sha256'], 'pipelined_steps': d['pipeline'].get('pipelined_steps'),
               'seq_ms': d['pipeline'].get('unpipelined_ms_per_step'),
               'probe_gbs': d.get('read_probe_gbs'), 'e2e': d.get('e2e_host_gibs'),
               'cpu': (d.get('cpu_baseline') or {}).get('value'),
               'warmup_steps': (d.get('warmup_run') or {}).get('steps')}
        print(json.dumps(out))


if __name__ == '__main__':
    main()

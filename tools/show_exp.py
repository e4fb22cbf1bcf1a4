import json, sys
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "missing", e); continue
    pk = d['extra']['per_kernel']
    par = (d['extra'].get('parity_vs_oracle') or {}).get('identical')
    print(f, d['value'], d['ms_per_step'], 'parity', par)
    print('   ', ' '.join('%s=%.3f' % (k, v['ms_per_step']) for k, v in pk.items() if v['ms_per_step'] > 0.04))

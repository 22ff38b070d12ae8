set -o pipefail
timeout -k 10 600 python -u bench.py --blocks 8 --block-size 25000 --K 1 --cpu-blocks 8 --read-bw 0 > gpurun_out/r03s6_c2val.json 2> gpurun_out/r03s6_c2val.err || { tail gpurun_out/r03s6_c2val.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03s6_c2val.json')); c=d['cpu_baseline']; print(d['value'], json.dumps({k:c[k] for k in c if k!='sample'}, indent=0)); print(c['sample'])"
timeout -k 10 600 python -u bench.py > gpurun_out/r03s6_ns.json 2> gpurun_out/r03s6_ns.err || { tail gpurun_out/r03s6_ns.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03s6_ns.json')); c=d['cpu_baseline']; print(d['value'], d['roofline']['frac'], json.dumps({k:c[k] for k in c if k!='sample'}, indent=0)); print(c['sample'])"

set -uo pipefail
mkdir -p gpurun_out/r06c
for u in 8192 16384 32768 65536; do for w in 768 1152; do
  CVD_CHUNK_UNITS=$u CVD_CHUNK_WARM=$w timeout -k 10 200 python3 profiles/r06_refcall.py --modes=-1 --early 0 --reps 3 > gpurun_out/r06c/u${u}_w${w}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r06c/u${u}_w${w}.json'));r=d['runs'][0];print($u,$w,[round(x,4) for x in r['seconds']],r['chunk_last'])"
done; done

for cfg in "1024 153600" "512 76800" "512 51200" "256 38400" "512 102400" "256 51200"; do
  set -- $cfg
  RURE_AMD_DEBUG=core_bs=$1,core_lds=$2 timeout -k 10 200 python bench.py --config c4 --no-cpu --steps 10 > gpurun_out/c4_$1_$2.json 2>&1 || exit 1
  echo "$1 $2 $(python -c "import json;d=json.loads(open('gpurun_out/c4_$1_$2.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['roofline']['kernel_ms'])")"
done

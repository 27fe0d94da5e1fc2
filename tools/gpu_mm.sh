cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for mm in 11 10 9; do
KC_SKM_MMIN=$mm KC_DEBUG=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/mm$mm.json 2> gpurun_out/mm$mm.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/mm$mm.json'));print($mm, round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],2),'ms',d['breakdown_ms_per_step']['partition_passes'])"
grep "kc: skm" gpurun_out/mm$mm.err | tail -2
done

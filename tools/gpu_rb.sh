cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in 2 1 2 1; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --wino-block1 $v > gpurun_out/rb_$v.log 2>&1 || exit $?
  python3 -c "
import json
s=open('gpurun_out/rb_$v.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
print('wb=$v', d['value'], d['ms_per_step'], 'p50', d['ms_per_clip_p50'], 'head', d['stage_ms']['head'], 'b2c1', d['stage_ms']['b2c1'], 'x3', d['value_x3']['value'])"
done

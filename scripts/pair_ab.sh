# Update passes paired (actor + critic same-shape layers per launch) vs separate: C3 and the 16384-env share.
set -e
mkdir -p gpurun_out/pab
for envs in ${PAB_ENVS:-16384 65536}; do
  for pt in ${PAB_PT:-0 1}; do
    RSLRL_PAIR_TRAIN=$pt timeout -k 10 200 python bench.py --global-num-envs $envs --no-extra --no-cpu-baseline --steps 20 > gpurun_out/pab/e${envs}_p$pt.json 2> gpurun_out/pab/e${envs}_p$pt.err
  done
done

# Same-box A/B of the staged permutation upload (RSLRL_STAGE_PERM=0 / 1) at the 16,384-env share and C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6stageab}
mkdir -p $o
for r in 1 2 3; do
  for f in 0 1; do
    for n in 16384 65536; do
      RSLRL_STAGE_PERM=$f timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_f${f}_r$r.json 2> $o/b${n}_f${f}_r$r.err || { tail -20 $o/b${n}_f${f}_r$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o/b${n}_f${f}_r$r.json'));print($n,'stage',$f,'run',$r,d['value'],d['ms_per_step'])"
    done
  done
done

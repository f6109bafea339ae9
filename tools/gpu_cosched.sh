# gen-kernel residency cap vs configs (C3, C4, C5-lite) and the 8-band rank launches
set -o pipefail
cd $GRAFT_REPO_ROOT
for cap in 0 3 4; do
  for cfg in C3 C4 C5; do
    RTMI_GEN_WAVES_CAP=$cap CONFIG=$cfg REPS=5 timeout -k 10 120 python tools/time_c3.py | cut -c1-110 || exit 1
  done
  RTMI_GEN_WAVES_CAP=$cap BANDS=4 REPS=5 timeout -k 10 200 python tools/scaling_sim.py || exit 1
done

# Standalone durations of the two-class launch's kernels (RTMI_SPLIT_SERIAL:
# both on one stream) next to the default concurrent launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/serial
mkdir -p $O
timeout -k 10 200 python tools/time_c3.py > $O/conc.json 2> $O/conc.err && \
RTMI_SPLIT_SERIAL=1 timeout -k 10 200 python tools/time_c3.py > $O/serial.json 2> $O/serial.err && \
RTMI_SPLIT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o s -f csv -- python3 tools/time_c3.py > /dev/null 2> $O/prof.err
rc=$?; cat $O/conc.json $O/serial.json; find $O/prof -name "*stats*" | xargs cat | head -8; exit $rc

set -o pipefail
bash tools/profile_round.sh &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "done $?"

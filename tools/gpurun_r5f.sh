# Round-5 tree on MI355X: 100-admission tail study (kfd open per slow step), then the
# native-daemon GPU tests under TSan and ASan/UBSan, then a 4-minute soak.
set -o pipefail
bash tools/gpurun_r5e.sh || exit 1
bash tools/gpurun_check.sh tsan asan soak

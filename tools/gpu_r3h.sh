set -e
bash tools/gpu_tests.sh
bash profiles/run_profile.sh r3d

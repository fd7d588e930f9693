set -o pipefail
bash tools/ab.sh orig main o3 orig main o3

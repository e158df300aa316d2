set -o pipefail
for cfg in "1024 4" "2048 4" "4096 8" "8192 16"; do set -- $cfg; OBST_MAP_WG=$1 OBST_MAP_SPLIT=$2 timeout -k 10 200 python -u tools/lab/attn_map_lab.py 2>&1 | grep fwd || exit 1; done

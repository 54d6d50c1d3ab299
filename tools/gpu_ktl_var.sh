# GPU box: serialized kernel timeline per library variant (VARS), decide kernels only
cd $GRAFT_REPO_ROOT
for v in ${VARS:-sentinel_flow}; do
echo "== $v"
SENTINEL_FLOW_LIB=$PWD/sentinel_amd/lib$v.so SF_SERIAL_STREAMS=1 NAME=ktl_$v bash tools/gpu_ktl.sh | grep -E "${PAT:-light|short|fill|stream|keys|unpack}" | tail -${TAILN:-8} || exit 1
done

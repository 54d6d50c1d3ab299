# A/B builds of the engine library with extra -D flags (diagnostics; not shipped):
#   bash tools/build_variants.sh name1="-DX=1" name2="-DY"   ->  sentinel_amd/variants/<name>.so
# select one at run time with SENTINEL_FLOW_LIB=sentinel_amd/variants/<name>.so
cd "$(dirname "$0")/../sentinel_amd/csrc" || exit 1
mkdir -p ../variants
pids=()
for kv in "$@"; do
  name=${kv%%=*}; flags=${kv#*=}
  make -s -j3 OUT=../variants/$name.so BUILD=build_v_$name EXTRA="$flags" > /tmp/bv_$name.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
ls -la ../variants
exit $rc

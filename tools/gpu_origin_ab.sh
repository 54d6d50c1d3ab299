# A/B of the wave walk variants (sentinel_amd/variants/<v>.so; "main" = the product library)
set -o pipefail
mkdir -p gpurun_out
for v in ${XW_VARIANTS:-prev main}; do
  if [ $v = main ]; then lib=""; else lib=sentinel_amd/variants/$v.so; fi
  SENTINEL_FLOW_LIB=$lib timeout -k 10 300 python3 -u tools/origin_ab.py other_rules_1pct 3 >> gpurun_out/oab.json 2>> gpurun_out/oab.err || exit 1
done

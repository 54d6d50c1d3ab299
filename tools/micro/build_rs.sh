# builds rsbench2 variants of the product sort (sf_rsort.h) for gfx950
cd "$(dirname "$0")"
for v in "8 8" "8 4"; do
  set -- $v
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-result -Wno-unused-value -DSF_RS_DB=$1 -DSF_RS_W=$2 -o rsb_$1_$2 rsbench2.hip &
done
wait

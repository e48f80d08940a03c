set -e
o=gpurun_out/sk3.txt; : > $o
for v in "" "SK_RR=8" "SK_NG=8" "SK_NG=8 SK_RR=8" "SK_NG=8 SK_BLOCKS=512" "SK_NG=8 SK_RR=8 SK_BLOCKS=512" "SK_BLOCKS=512" "SK_RR=8 SK_BLOCKS=512"; do
  echo "== $v" >> $o
  env $v timeout -k 10 60 ./tools/skinny_bench >> $o 2>&1
done

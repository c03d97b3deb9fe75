# diagnostics: config-5 C3 time of the library variants under lib/variants (tools/build_variant.sh)
set -e
mkdir -p gpurun_out
for v in base $(cd mapping-private_amd/lib/variants && ls *.so | sed 's/\.so$//'); do
  if [ $v = base ]; then L=mapping-private_amd/lib/libc3hlac_mi355x.so; else L=mapping-private_amd/lib/variants/$v.so; fi
  echo "== $v"
  C3HLAC_LIB=$L timeout -k 10 240 python -u tools/config5.py > gpurun_out/mfexp_$v.log 2>&1
  grep -E "rep 3" gpurun_out/mfexp_$v.log
done

# round 3: march low-transmittance schedule sweep around the default (k_low 8, t_split 0.9, growth from round 8)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for dt in bf16 fp32; do
  timeout -k 10 300 python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9_g8,12x2_klow8_t0.7_g8,12x2_klow8_t0.5_g8,12x2_klow16_t0.9_g8,12x2_klow16_t0.7_g8,12x2_klow4_t0.9_g8,12x2_klow8_t0.9_g6,12x2_klow8_t0.9_g10 > gpurun_out/march_sweep4_$dt.json 2> gpurun_out/march_sweep4_$dt.log
  r=$?; echo "$dt rc=$r"; cat gpurun_out/march_sweep4_$dt.json; if [ $r -ne 0 ]; then exit $r; fi
done

set -u
bash tools/gpu_profile.sh r04f_cfg5 --workload cfg5_100k_60x_ul_ont && \
bash tools/gpu_profile.sh r04f_cfg3 --workload cfg3_50k_delins_30x_ont && \
bash tools/gpu_profile.sh r04f_cfg2 --workload cfg2_10kdel_30x_ont && \
bash tools/gpu_profile.sh r04f_cfg1 --workload cfg1_100del_10x && \
bash tools/gpu_steps.sh r04_infab 'inf_old|300|SVTREK_ENGINE_LIB=$PWD/variants/a_inf_old.so python tools/bench_inflate.py --scale 0.1 --reps 3' 'inf_new|300|SVTREK_ENGINE_LIB=$PWD/variants/b_inf_vwin.so python tools/bench_inflate.py --scale 0.1 --reps 3'

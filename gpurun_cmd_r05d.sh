# Evidence at HEAD: rocprofv3 kernel stats + HBM traffic of the default bench launch (C3), kernel
# stats of the C2 and C4 rows, then the default bench line.
bash scripts/steps.sh r05d \
 "prof_c3|500|TAG=r05d STEPS=5 bash scripts/profile.sh && python scripts/summarize_profile.py gpurun_out/prof_r05d r05d" \
 "prof_c2|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_r05d_c2 -o run -- python3 \$GRAFT_REPO_ROOT/bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline" \
 "prof_c4|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_r05d_c4 -o run -- python3 \$GRAFT_REPO_ROOT/bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline" \
 "bench|300|python bench.py"

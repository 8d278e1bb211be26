export AB_NAME0=r01 AB_NAME1=head AB_NAME2=head AB_NAME3=r01
tools/gpurun/steps.sh \
 "120 abfold1 ./tools/abtest/ab_fold 10000000 9" \
 "240 bench_head python3 -u bench.py --no-cpu-baseline --no-e2e --no-extras --steps 20 --warmup 3" \
 "240 bench_r01 cd tools/abtest/r01tree && python3 -u bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3" \
 "120 abfold2 ./tools/abtest/ab_fold 10000000 9"

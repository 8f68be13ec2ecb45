export TMPDIR=/tmp; mkdir -p gpurun_out/r04d
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04d/bench.json 2> gpurun_out/r04d/bench.err || { tail -20 gpurun_out/r04d/bench.err; exit 1; }
tail -c 300 gpurun_out/r04d/bench.json
bash scripts/ab_tune.sh gpurun_out/r04d/ab_net - "--crc --corrupt none --steps 10 --warmup 3 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample" new= old=@hdfs-native_amd/lib/libhdfs_ec_amd_exp.so new2= old2=@hdfs-native_amd/lib/libhdfs_ec_amd_exp.so || exit 2
bash scripts/pmc_verify.sh gpurun_out/r04d/pmcv || exit 3
timeout -k 10 1200 python3 -u scripts/profile_configs.py gpurun_out/r04d/prof crc63 > gpurun_out/r04d/prof.log 2>&1; tail -5 gpurun_out/r04d/prof.log

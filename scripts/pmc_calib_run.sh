set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/cal_w -o run --output-format csv -- python3 scripts/pmc_calib.py 5 > gpurun_out/pmc/cal_w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/cal_f -o run --output-format csv -- python3 scripts/pmc_calib.py 5 > gpurun_out/pmc/cal_f.log 2>&1
PMC_SCENE=committed timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/com_w -o run --output-format csv -- python3 scripts/pmc_workload.py 5 > gpurun_out/pmc/com_w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/fac_w -o run --output-format csv -- python3 scripts/pmc_workload.py 5 > gpurun_out/pmc/fac_w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fac_f -o run --output-format csv -- python3 scripts/pmc_workload.py 5 > gpurun_out/pmc/fac_f.log 2>&1
echo pmc done

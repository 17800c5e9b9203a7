# FETCH_SIZE / WRITE_SIZE calibration (tools/probe/fetch_calib.hip): one PMC
# pass each, outputs under gpurun_out/calib_*; summarised by
# tools/probe/calib_summary.py into profiles/r06_fetch_calibration.json
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o pmc -- ./tools/probe/fetch_calib > gpurun_out/calib_fetch.log 2>&1 || { echo calib fetch failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o pmc -- ./tools/probe/fetch_calib > gpurun_out/calib_write.log 2>&1 || { echo calib write failed; exit 1; }
echo CALIB_DONE

#!/bin/bash
# Round-3 pass A: new ECoG / index / packed-export tests, then the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_ecog.py "tests/test_gpu_api.py::test_compute_elbo_unsorted_index_matches_oracle" \
  "tests/test_gpu_training_api.py::test_packed_export_allocates_no_device_memory" \
  "tests/test_gpu_training_api.py::test_packed_pair_layout_matches_dense" \
  "tests/test_gpu_pair_shard.py::test_two_rank_pair_sharded_training" \
  -x -v -s --timeout 900 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r03a_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
rc2=$?
tail -1 gpurun_out/r03a_bench.json | cut -c1-400
exit $(( rc | rc2 ))

set -e
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNMGP_BIG_TRACE -Icollaborative_nonstationary_multivariate_gaussian_process_amd/csrc -Iinclude tools/big_trace.hip -o /tmp/big_trace 2>/dev/null
for c in "128 128 512 0" "128 128 512 1" "3584 128 512 1" "3584 128 512 0" "3072 3072 512 0" "3840 3840 128 1" "128 128 4096 0"; do
  timeout -k 5 30 /tmp/big_trace $c
done

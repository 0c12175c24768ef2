set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_vm.py tests/test_gpu_http.py tests/test_gpu_http_map.py "tests/test_gpu_parity.py::test_utf8_validation_pinned_to_reference_validator" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprofns.so DG_ALLOW_STALE=1 timeout -k 10 120 python tools/flprof.py c2 > $O/phases_nostore_c2.txt 2>&1 && DG_LIB_PATH=dynamicgo_amd/libdgj2t_wprof.so DG_ALLOW_STALE=1 timeout -k 10 200 python tools/wprof.py c3 > $O/wprof_c3.txt 2>&1; grep -v amdgpu.ids $O/*.txt

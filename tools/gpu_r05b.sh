set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r05b
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py tests/test_jni_shim.py -m gpu -x -q --timeout 200 --timeout-method thread -k "overlapped or config3 or fwt2d or config2 or fwt_large or chain or in_place or host_entry or multi or drop_in" > gpurun_out/r05b/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05b/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05b/pytest.log | head; exit 1; }
L=jwave_amd/lib
bash tools/gpu_ab_libs.sh fwt2d 3 $L/ab_ser.so $L/libjwave_hip.so $L/ab_g8.so $L/ab_np.so $L/ab_g2.so

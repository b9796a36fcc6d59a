export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/fullframe_outliers.py > gpurun_out/ff_outliers.log 2>&1 || { echo ff failed; tail -20 gpurun_out/ff_outliers.log; exit 1; }
tail -12 gpurun_out/ff_outliers.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_abi.py tests/test_gpu_kernels.py -k "abi or composite_pdf" > gpurun_out/t_abi_cpdf.log 2>&1 || { echo tests failed; tail -30 gpurun_out/t_abi_cpdf.log; exit 1; }
tail -3 gpurun_out/t_abi_cpdf.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_training.py -k psnr > gpurun_out/t_psnr.log 2>&1 || { echo psnr failed; tail -30 gpurun_out/t_psnr.log; exit 1; }
grep PSNR gpurun_out/t_psnr.log | cut -c1-1500; tail -3 gpurun_out/t_psnr.log

cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/nk_base_$i.log 2>&1; echo "base $(tail -1 gpurun_out/nk_base_$i.log | cut -c1-200)"
  HIPFM_KERNELS_SO=$GRAFT_REPO_ROOT/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib/libhipfm_kernels_nk.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/nk_var_$i.log 2>&1; echo "noklp $(tail -1 gpurun_out/nk_var_$i.log | cut -c1-200)"
done

# lab A/B: libsmfv_lab.so (SMFV_LAB=1, built from a modified copy of the kernels) vs libsmfv.so
AB_LIST="SMFV_LAB=1;SMFV_LAB=0;SMFV_LAB=1;SMFV_LAB=0;SMFV_LAB=1;SMFV_LAB=0" TAG=${TAG:-ab} bash scripts/gpu_ab_env.sh || exit 1
AB_ARGS="--config cop20k_k128" AB_LIST="SMFV_LAB=1;SMFV_LAB=0;SMFV_LAB=1;SMFV_LAB=0" TAG=${TAG:-ab}_k128 bash scripts/gpu_ab_env.sh

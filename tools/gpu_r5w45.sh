# r5w4 then r5w5 in one call
bash tools/gpu_r5w4.sh r5w4 && bash tools/gpu_r5w5.sh r5w5

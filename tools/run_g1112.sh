# GPU box: g11 (windowed SpMV pipelining, CG) then g12 (k_line2 four levels per step)
bash tools/run_g11.sh && bash tools/run_g12.sh

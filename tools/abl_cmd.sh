mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_gen.py -q -x > gpurun_out/t_gen.log 2>&1 || { tail -20 gpurun_out/t_gen.log; exit 1; }
( timeout -k 10 60 python tools/kbench.py
for A in 1 2 4 8 16 32 64 31 96; do LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_abl$A.so timeout -k 10 60 python tools/kbench.py || exit 1; done ) > gpurun_out/abl.jsonl 2> gpurun_out/abl.err
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --gen-seconds 1 > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err

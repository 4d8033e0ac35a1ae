timeout -k 10 120 python scripts/wbw.py > gpurun_out/wbw.json 2>&1

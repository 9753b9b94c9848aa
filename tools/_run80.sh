timeout -k 10 120 python tools/fused_check.py

source scripts/gpu/guard.sh
step dbg timeout -k 10 120 python scripts/debug/coho_debug2.py

set -u
timeout -k 10 300 python scripts/r04_ragged_probe.py && TONEHIP_LIB=t-one_amd/libtonehip_base.so timeout -k 10 300 python scripts/r04_ragged_probe.py

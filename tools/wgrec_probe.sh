for o in 0 1; do
CTOK_WGREC=1 CTOK_OVERLAP=$o timeout -k 10 300 python -u tools/probe.py C4S8 gpt2_50k 2 2>&1 | grep -E "wgrec|MB/s" | tail -5
CTOK_WGREC=1 CTOK_OVERLAP=$o timeout -k 10 300 python -u tools/probe.py C4 gpt2_50k 2 2>&1 | grep -E "wgrec|MB/s" | tail -5
done

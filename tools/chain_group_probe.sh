B=tools/bin/bench_chain_base_ar
for d in 0 1; do
  for n in 2 64 128 256; do DISTINCT_RECS=$d timeout -k 5 60 $B 400 0 time $n | head -1 | sed "s/^/d=$d /" || exit 1; done
  DISTINCT_RECS=$d CHAIN_LDS_BYTES=80896 timeout -k 5 60 $B 400 0 time 512 | head -1 | sed "s/^/d=$d lds80k /" || exit 1
  DISTINCT_RECS=$d CHAIN_LDS_BYTES=39936 timeout -k 5 60 $B 400 0 time 1024 | head -1 | sed "s/^/d=$d lds40k /" || exit 1
done

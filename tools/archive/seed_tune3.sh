# pass-1 slice capacities: mems / chains raised (host overflow histogram: MEMS 2.8 %, CHAINS 0.4 % of reads at 256/256)
mkdir -p gpurun_out
run() { PRGPU_SEED_WAVES_PER_CU=$1 PRGPU_SEED_SMALL=$2 timeout -k 10 300 python -u tools/seed_time.py >> gpurun_out/seedtune3.log 2>&1; }
run 16 4096,64,256,512,256 && run 16 4096,64,512,512,384 && run 16 4096,64,512,512,256 && run 16 4096,64,384,512,384 && run 16 4096,64,640,640,448

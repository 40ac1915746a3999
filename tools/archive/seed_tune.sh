# tuning sweep of the GPU seeding pass 1 (waves per CU, small-slice capacities)
mkdir -p gpurun_out
run() { PRGPU_SEED_WAVES_PER_CU=$1 PRGPU_SEED_SMALL=$2 timeout -k 10 300 python -u tools/seed_time.py >> gpurun_out/seedtune2.log 2>&1; }
run 16 4096,64,256,512,256 && run 8 8192,64,256,512,256 && run 8 8192,128,512,1024,512 && run 12 8192,64,256,1024,256 && run 16 6144,64,256,768,256

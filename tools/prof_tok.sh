set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
timeout -k 10 300 python tools/tok_perf.py 128 > gpurun_out/prof1/perf.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/kt -o kt --output-format csv -- python tools/tok_perf.py 64 > gpurun_out/prof1/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/prof1/pmc1 -o pmc1 --output-format csv -- python tools/tok_perf.py 64 > gpurun_out/prof1/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/prof1/pmc2 -o pmc2 --output-format csv -- python tools/tok_perf.py 64 > gpurun_out/prof1/pmc2.log 2>&1
cat gpurun_out/prof1/perf.txt

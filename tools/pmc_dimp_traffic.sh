# HBM traffic of the mfDiMP bench's feature net: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 PMC passes
set -e
OUT=${OUT:-gpurun_out/pmc_dimp_traffic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--workload mfdimp_rgbt --batch 32 --steps 3 --warmup 1 --no-cpu-baseline --sync"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python bench.py $ARGS > $OUT/write.log 2>&1
ALG=$(python -c "
import sys; sys.path.insert(0, 'multi-modal-trakcing-bechmark_amd')
from mmtrack_amd import synth
from mmtrack_amd.dimpnet import DiMPNet
net = DiMPNet(synth.make_dimp_state_dict(0))
print(32 * sum(b for _, b in net.layer_work()))")
python tools/pmc_dimp_traffic.py $OUT ${DEST:-$OUT/pmc_traffic_dimp.json} $ALG

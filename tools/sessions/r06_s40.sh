# gradient batch jobs longest first vs call order: step A/B on one box (interleaved, x2)
export TMPDIR=/tmp
STEPS=200 bash tools/gpu_lib_ab.sh r06_s40 2 main noord || exit $?

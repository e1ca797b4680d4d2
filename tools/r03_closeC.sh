# round-3 closing set (second session): parts A and B in one call
set -o pipefail
bash tools/r03_closeA.sh ${1:-r03_close2} || exit $?
bash tools/r03_closeB.sh ${1:-r03_close2} || exit $?

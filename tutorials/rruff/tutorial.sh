#!/bin/bash
# RRUFF powder-XRD tutorial: pdif turns DIF + raw XY records into samples
# (850 intensity bins + temperature -> 230 space groups, ANN), then train_nn / run_nn.
# Workflow of the reference's tutorials/ann/tutorial.bash, non-interactive and offline:
# records are read from $RRUFF_DIR/{dif,raw} (default ./rruff); without them a
# synthetic RRUFF-shaped set is generated (hpnn_amd.utils.synth, NREC records).
#
# Environment: NREC=400  HIDDEN=200  PASSES=3  MODE=batched|online  BATCH=16
#              EPOCHS=50  WORK=./rruff_run  FLAGS (extra train_nn/run_nn flags)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$HERE/../..
BIN=${BIN:-$ROOT/bin}
for t in pdif train_nn run_nn; do
  [ -x "$BIN/$t" ] || { echo "missing $BIN/$t (run make first)"; exit 1; }
done
NREC=${NREC:-400}; HIDDEN=${HIDDEN:-200}; PASSES=${PASSES:-3}; MODE=${MODE:-batched}
BATCH=${BATCH:-16}; EPOCHS=${EPOCHS:-50}; WORK=${WORK:-./rruff_run}; RRUFF_DIR=${RRUFF_DIR:-./rruff}
mkdir -p "$WORK"; WORK=$(cd "$WORK" && pwd)
if [ ! -d "$RRUFF_DIR/dif" ]; then
  echo "no RRUFF records in $RRUFF_DIR: generating $NREC synthetic records"
  RRUFF_DIR=$WORK/rruff
  PYTHONPATH=$ROOT${PYTHONPATH:+:$PYTHONPATH} python3 -m hpnn_amd.utils.synth "$RRUFF_DIR" -n "$NREC"
fi
rm -rf "$WORK/samples" "$WORK/tests"; mkdir -p "$WORK/samples" "$WORK/tests"
"$BIN/pdif" "$RRUFF_DIR" -i 850 -o 230 -s "$WORK/samples" | tail -1
cd "$WORK"
# hold out every 10th sample as the test set
ls samples | awk 'NR % 10 == 0' | while read -r f; do mv "samples/$f" tests/; done
EXTRA=""
[ "$MODE" = batched ] && EXTRA="[mode] batched
[batch] $BATCH
[epochs] $EPOCHS"
cat > rruff.conf <<!
[name] RRUFF
[type] ANN
[init] generate
[seed] 10958
[input] 851
[hidden] $HIDDEN
[output] 230
[train] BPM
[sample_dir] ./samples
[test_dir] ./tests
$EXTRA
!
sed -e 's/^\[init\].*/[init] kernel.opt/' -e 's/^\[seed\].*/[seed] 0/' rruff.conf > cont_rruff.conf
: > raw
for P in $(seq 1 "$PASSES"); do
  CONF=cont_rruff.conf; [ "$P" = 1 ] && CONF=rruff.conf
  "$BIN/train_nn" -v -v $FLAGS "$CONF" > log 2>&1
  "$BIN/run_nn" -v $FLAGS cont_rruff.conf > results 2>&1
  ACC=$(grep ACCURACY results | awk '{split($2, a, "/"); printf "%.1f", 100 * a[1] / a[2]}')
  echo "$P $ACC" | tee -a raw
done
echo "All DONE! (pass test-accuracy[%] in $WORK/raw)"

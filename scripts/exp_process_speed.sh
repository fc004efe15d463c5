#!/bin/bash
# Is the 7 % spread between runs of identical code a property of the process or of the moment?
# N processes back to back, each building the bench graph and timing three runs of 20 rounds.
# usage: scripts/exp_process_speed.sh N
for i in $(seq $1); do
  echo "process $i at $(date +%H:%M:%S.%N | cut -c1-12)"
  timeout -k 10 200 scripts/probes/lib_ab page-rank-and-tfidf-using-apache-spark_amd/_build/libprmi355x.so 26 20 3 | sed 's/page-rank-and-tfidf-using-apache-spark_amd\/_build\///' || exit 1
done

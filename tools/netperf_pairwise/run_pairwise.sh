#!/bin/sh
# One iperf3 -J report per ordered node pair: <client hostIP>_<server hostIP>.json,
# copied into the scheduler pod's /home like the reference's run.sh:3-14 does
# for its star.  The host mirror reads them with nas_host_latency_matrix
# (include/nas_host.h) -- the same Go json semantics as scheduler.go:503-530 --
# and uploads the resulting N x N matrix once (nas_upload_latency).
# Usage: ./run_pairwise.sh [extra iperf3 client args, e.g. -t 5]
set -eu
CLIENTS=$(kubectl get pods -l app=iperf3-pair-client -o name | cut -d'/' -f2)
SERVERS=$(kubectl get pods -l app=iperf3-pair-server -o jsonpath='{range .items[*]}{.status.hostIP},{.status.podIP}{"\n"}{end}')
SCHEDULER=$(kubectl get pods -l app=custom-scheduler -o name | cut -d'/' -f2)
for POD in ${CLIENTS}; do
    until [ "$(kubectl get pod "${POD}" -o jsonpath='{.status.containerStatuses[0].ready}')" = "true" ]; do
        echo "Waiting for ${POD} to start..."
        sleep 5
    done
    CHOST=$(kubectl get pod "${POD}" -o jsonpath='{.status.hostIP}')
    for S in ${SERVERS}; do
        SHOST=${S%,*}
        SIP=${S#*,}
        [ "${SHOST}" = "${CHOST}" ] && continue
        OUT="${CHOST}_${SHOST}.json"
        # one pair at a time: concurrent tests would share links and skew each other
        kubectl exec "${POD}" -- iperf3 -c "${SIP}" -Z -J -T "Client on ${CHOST}" "$@" > "${OUT}.tmp" || true
        mv "${OUT}.tmp" "${OUT}"
        kubectl cp "${OUT}" "${SCHEDULER}:/home"
    done
done

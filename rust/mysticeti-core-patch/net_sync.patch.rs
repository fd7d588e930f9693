// NetworkSyncer::process_blocks (mysticeti-core/src/net_sync.rs:314-386) with the GPU engine.
// Order kept from the reference:
//   1. `processed` is fetched for the whole message (net_sync.rs:325-328);
//   2. blocks already processed are skipped BEFORE any verification (net_sync.rs:331-335) --
//      so they are filtered out before the batch call, not verified and then dropped;
//   3. per remaining block, in message order: the consensus-rule verdict (now precomputed by
//      one batch call), then the custom BlockVerifier; the first failure ends the connection.
async fn process_blocks(
    inner: &Arc<NetworkSyncerInner<H, C>>,
    block_verifier: &Arc<impl BlockVerifier>,
    metrics: &Arc<Metrics>,
    blocks: Vec<Data<StatementBlock>>,
) -> Result<Vec<BlockReference>, eyre::Report> {
    if blocks.is_empty() {
        return Ok(vec![]);
    }
    let now = timestamp_utc();
    let processed = inner
        .syncer
        .processed(blocks.iter().map(|block| *block.reference()).collect())
        .await;
    let fresh: Vec<Data<StatementBlock>> =
        blocks.into_iter().filter(|b| !processed.contains(b.reference())).collect();
    for b in &fresh {
        tracing::debug!("Received {} from {}", b.reference(),
                        inner.committee.authority_safe(b.author()).hostname());
    }
    // one engine call for the message; spawn_blocking keeps the tokio worker free, and the
    // engine's submission queue merges concurrent peers' calls into one GPU pass
    let verdicts = tokio::task::spawn_blocking({
        let gpu = inner.gpu_verifier.clone(); // Arc<GpuVerifier>
        let committee = inner.committee.clone();
        let fresh = fresh.clone();
        move || gpu.verify_blocks(&fresh, &committee)
    })
    .await?;

    let mut to_process = Vec::new();
    for (block, verdict) in fresh.into_iter().zip(verdicts) {
        let hostname = inner.committee.authority_safe(block.author()).hostname();
        metrics
            .block_receive_latency
            .with_label_values(&[&hostname])
            .observe(now.checked_sub(block.meta_creation_time()).unwrap_or_default().as_secs_f64());
        if let Err(e) = verdict {
            tracing::warn!("Rejected incorrect block {} based on consensus rules from {}: {:?}",
                           block.reference(), hostname, e);
            return Err(e); // terminate the connection, as net_sync.rs:352-361
        }
        if let Err(e) = block_verifier.verify(&block).await {
            tracing::warn!("Rejected incorrect block {} based on validation rules from {}: {:?}",
                           block.reference(), hostname, e);
            return Err(eyre::Report::msg(""));
        }
        to_process.push(block);
    }
    if !to_process.is_empty() {
        let connected_authorities = inner.connected_authorities.lock().authorities.clone();
        return Ok(inner.syncer.add_blocks(to_process, connected_authorities).await);
    }
    Ok(vec![])
}

/*
 * The gossip signature service on the GPU backend: AggregatingSignatureVerificationService
 * (ethereum/statetransition/.../validation/signatures/AggregatingSignatureVerificationService.java)
 * with three changes, the rest (queue, capacity error, metrics, waitForBatch)
 * kept as the reference has it.
 *  1. Workers: one per device (HipBatchVerifier.deviceCount()), where the
 *     reference sizes numThreads to the host cores (l.68-69; P2PConfig.java:42-43).
 *  2. batchVerifySignatures: the batch and, when it fails, every set's
 *     verdict in ONE device call (tbls_batch_verify_each), instead of
 *     BLS.batchVerify plus the recursive halving and per-task SIMPLE.verify of
 *     l.202-226.  A task is valid iff all its sets are (BLSSignatureVerifier
 *     .SIMPLE.verify -> BLS.batchVerify over the task's sets,
 *     BLSSignatureVerifier.java:27-43: the same boolean with overwhelming
 *     probability).
 *  3. Placement: a worker whose batch leaves tasks waiting in the queue asks
 *     for one device (nGpus = 1), so concurrent batches run on distinct
 *     devices; a batch that drains the queue may shard over every idle
 *     device (tb_lib.hip place_plan: down to 4,096 sets per device on an
 *     idle node).
 * Python mirror and tests: teku_amd/service.py, tests/test_service.py
 * (placement simulated over 8 devices), tests/test_gpu_configs.py.
 */
package tech.pegasys.teku.statetransition.validation.signatures;

import static java.util.Collections.singletonList;

import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.ArrayBlockingQueue;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.TimeUnit;
import org.apache.logging.log4j.LogManager;
import org.apache.logging.log4j.Logger;
import org.apache.tuweni.bytes.Bytes;
import org.hyperledger.besu.plugin.services.MetricsSystem;
import org.hyperledger.besu.plugin.services.metrics.Counter;
import tech.pegasys.teku.bls.BLSPublicKey;
import tech.pegasys.teku.bls.BLSSignature;
import tech.pegasys.teku.bls.impl.hip.HipBatchVerifier;
import tech.pegasys.teku.infrastructure.async.AsyncRunner;
import tech.pegasys.teku.infrastructure.async.AsyncRunnerFactory;
import tech.pegasys.teku.infrastructure.async.SafeFuture;
import tech.pegasys.teku.infrastructure.metrics.MetricsHistogram;
import tech.pegasys.teku.infrastructure.metrics.TekuMetricCategory;
import tech.pegasys.teku.service.serviceutils.ServiceCapacityExceededException;

public class HipAggregatingSignatureVerificationService extends SignatureVerificationService {
  private static final Logger LOG = LogManager.getLogger();

  /* the device wants >= 16k sets per batch; the reference default is 250 */
  public static final int DEFAULT_MAX_BATCH_SIZE = 16384;

  private final AsyncRunner completionRunner;
  private final int numThreads;
  private final int maxBatchSize;
  private final BlockingQueue<Task> queue;
  private final AsyncRunner asyncRunner;
  private final Counter batchCounter;
  private final Counter taskCounter;
  private final MetricsHistogram batchSizeHistogram;

  public HipAggregatingSignatureVerificationService(
      final MetricsSystem metricsSystem,
      final AsyncRunnerFactory asyncRunnerFactory,
      final AsyncRunner completionRunner,
      final int queueCapacity,
      final int maxBatchSize) {
    this.numThreads = HipBatchVerifier.deviceCount();
    this.asyncRunner = asyncRunnerFactory.create(getClass().getSimpleName(), numThreads);
    this.completionRunner = completionRunner;
    this.maxBatchSize = maxBatchSize;
    this.queue = new ArrayBlockingQueue<>(queueCapacity);
    metricsSystem.createGauge(
        TekuMetricCategory.EXECUTOR,
        "signature_verifications_queue_size",
        "Tracks number of signatures waiting to be batch verified",
        queue::size);
    batchCounter =
        metricsSystem.createCounter(
            TekuMetricCategory.EXECUTOR,
            "signature_verifications_batch_count_total",
            "Reports the number of verification batches processed");
    taskCounter =
        metricsSystem.createCounter(
            TekuMetricCategory.EXECUTOR,
            "signature_verifications_task_count_total",
            "Reports the number of individual verification tasks processed");
    batchSizeHistogram =
        MetricsHistogram.create(
            TekuMetricCategory.EXECUTOR,
            metricsSystem,
            "signature_verifications_batch_size",
            "Histogram of signature verification batch sizes",
            3,
            List.of());
  }

  @Override
  protected SafeFuture<?> doStart() {
    for (int i = 0; i < numThreads; i++) {
      asyncRunner
          .runAsync(this::run)
          .finish(err -> LOG.error("GPU signature verification worker failed", err));
    }
    return SafeFuture.COMPLETE;
  }

  @Override
  protected SafeFuture<?> doStop() {
    return SafeFuture.COMPLETE;
  }

  @Override
  public SafeFuture<Boolean> verify(
      final List<BLSPublicKey> publicKeys, final Bytes message, final BLSSignature signature) {
    return verify(singletonList(publicKeys), singletonList(message), singletonList(signature));
  }

  @Override
  public SafeFuture<Boolean> verify(
      final List<List<BLSPublicKey>> publicKeys,
      final List<Bytes> messages,
      final List<BLSSignature> signatures) {
    assertIsRunning("verify");
    final Task task = new Task(completionRunner, publicKeys, messages, signatures);
    if (publicKeys.size() != messages.size() || messages.size() != signatures.size()) {
      task.result.completeExceptionally(new IllegalArgumentException("Different collection sizes"));
    } else if (!queue.offer(task)) {
      task.result.completeExceptionally(
          new ServiceCapacityExceededException("Failed to process signature, queue is full."));
    }
    return task.result;
  }

  private void run() {
    while (isRunning()) {
      final List<Task> tasks = new ArrayList<>();
      try {
        final Task first = queue.poll(30, TimeUnit.SECONDS);
        if (first != null) {
          tasks.add(first);
          queue.drainTo(tasks, maxBatchSize - 1);
        }
      } catch (InterruptedException e) {
        Thread.currentThread().interrupt();
      }
      if (!tasks.isEmpty()) {
        batchVerifySignatures(tasks);
      }
    }
  }

  void batchVerifySignatures(final List<Task> tasks) {
    batchCounter.inc();
    taskCounter.inc(tasks.size());
    batchSizeHistogram.recordValue(tasks.size());
    final List<List<BLSPublicKey>> allKeys = new ArrayList<>();
    final List<Bytes> allMessages = new ArrayList<>();
    final List<BLSSignature> allSignatures = new ArrayList<>();
    for (Task task : tasks) {
      allKeys.addAll(task.publicKeys);
      allMessages.addAll(task.messages);
      allSignatures.addAll(task.signatures);
    }
    final boolean[] okPerSet = new boolean[allKeys.size()];
    final int nGpus = queue.isEmpty() ? 0 : 1;
    final boolean batchIsValid;
    try {
      batchIsValid =
          allKeys.isEmpty()
              || HipBatchVerifier.batchVerifyEach(allKeys, allMessages, allSignatures, nGpus, okPerSet);
    } catch (RuntimeException e) {
      for (Task task : tasks) {
        task.result.completeExceptionally(e);
      }
      return;
    }
    int k = 0;
    for (Task task : tasks) {
      boolean valid = !task.publicKeys.isEmpty(); // SIMPLE.verify of no sets is false (BLS.java:240-241)
      for (int j = 0; j < task.publicKeys.size(); j++) {
        valid &= batchIsValid || okPerSet[k + j];
      }
      k += task.publicKeys.size();
      task.completeAsync(valid);
    }
  }

  static class Task {
    final SafeFuture<Boolean> result = new SafeFuture<>();
    private final AsyncRunner asyncRunner;
    final List<List<BLSPublicKey>> publicKeys;
    final List<Bytes> messages;
    final List<BLSSignature> signatures;

    Task(
        final AsyncRunner asyncRunner,
        final List<List<BLSPublicKey>> publicKeys,
        final List<Bytes> messages,
        final List<BLSSignature> signatures) {
      this.asyncRunner = asyncRunner;
      this.publicKeys = publicKeys;
      this.messages = messages;
      this.signatures = signatures;
    }

    void completeAsync(final boolean isValid) {
      asyncRunner.runAsync(() -> result.complete(isValid)).finish(result::completeExceptionally);
    }
  }
}

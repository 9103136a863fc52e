/*
 * HipNative — JNI entry points of libjwave_hip_jni.so (java/native/jwave_hip_jni.c),
 * a thin shim over the C ABI of libjwave_hip.so (include/jwave_hip.h).
 *
 * Source-only in this repository: the build image has no JDK (DESIGN.md §3).
 */
package jwave.amd;

import jwave.exceptions.JWaveError;
import jwave.exceptions.JWaveException;
import jwave.exceptions.JWaveFailure;
import jwave.transforms.wavelets.Wavelet;
import jwave.transforms.wavelets.biorthogonal.BiOrthogonal;
import jwave.transforms.wavelets.haar.Haar1Orthogonal;

public final class HipNative {

  static { System.loadLibrary( "jwave_hip_jni" ); }

  private HipNative( ) { }

  // status codes of include/jwave_hip.h
  static final int OK = 0, FAILURE = 1, ILLEGAL_ARGUMENT = 2, DEVICE = 3, BAD_CALL = 4;

  // one jwv_ctx per Java thread (the C ABI serialises per context; the
  // reference transforms are used concurrently: ParallelTransform.java:258-270)
  private static final ThreadLocal< Long > CTX = ThreadLocal.withInitial( ( ) -> {
    long[ ] h = new long[ 1 ];
    int rc = ctxCreate( Integer.getInteger( "jwave.hip.device", 0 ), h );
    if( rc != OK )
      throw new IllegalStateException( lastError( 0L ) );
    return h[ 0 ];
  } );

  static long ctx( ) { return CTX.get( ); }

  // Multi-device batches: -Djwave.hip.devices=0,1,...,7 spreads the batched
  // entries (forwardBatch / reverseBatch) over those GPUs, one contiguous
  // block of signals per device (jwv_mctx, include/jwave_hip.h), as the
  // reference's executor spreads independent signals over threads
  // (src/test/java/jwave/ParallelizationOpportunityTest.java:80-98).  Unset
  // or one device: the calling thread's single-device context.  One
  // multi-context per process (its calls are serialised; each runs one host
  // thread per device).
  private static long MCTX = -1L;
  // A bad jwave.hip.devices (unparsable, or a device the runtime rejects) is
  // remembered and rethrown on every batch call: the setting never falls back
  // to one device silently after its first failure.
  private static String MCTX_ERROR = null;

  static synchronized long mctx( ) {
    if( MCTX_ERROR != null )
      throw new IllegalStateException( MCTX_ERROR );
    if( MCTX >= 0 )
      return MCTX;
    String p = System.getProperty( "jwave.hip.devices" );
    if( p == null || p.trim( ).isEmpty( ) )
      return MCTX = 0L;
    String[ ] parts = p.trim( ).split( "\\s*,\\s*" );
    if( parts.length < 2 )
      return MCTX = 0L;
    int[ ] dev = new int[ parts.length ];
    try {
      for( int i = 0; i < dev.length; i++ )
        dev[ i ] = Integer.parseInt( parts[ i ] );
    } catch( NumberFormatException e ) {
      MCTX_ERROR = "jwave.hip.devices: not a device list: " + p;
      throw new IllegalStateException( MCTX_ERROR );
    }
    long[ ] h = new long[ 1 ];
    int rc = mctxCreate( dev, h );
    if( rc != OK ) {
      MCTX_ERROR = "jwave.hip.devices=" + p + ": " + mctxLastError( 0L );
      throw new IllegalStateException( MCTX_ERROR );
    }
    MCTX = h[ 0 ];
    return MCTX;
  }

  static void checkMulti( long m, int rc ) throws JWaveException {
    if( rc == OK )
      return;
    String msg = mctxLastError( m );
    switch( rc ) {
      case FAILURE:          throw new JWaveFailure( msg );
      case ILLEGAL_ARGUMENT: throw new IllegalArgumentException( msg );
      default:               throw new JWaveError( msg );
    }
  }

  /** Every row of m (equal lengths) with the same level in one native call:
   *  over the jwave.hip.devices GPUs when set, else this thread's device. */
  static double[ ][ ] batch( int kind, Taps t, boolean fwd, double[ ][ ] m, int level )
      throws JWaveException {
    int rows = m.length, cols = rows == 0 ? 0 : m[ 0 ].length;
    double[ ] x = pack( m ), y = new double[ x.length ];
    long mc = mctx( );
    if( mc != 0L )
      checkMulti( mc, transformBatchMulti( mc, kind, fwd, x, y, rows, cols, level, t.L, t.tw,
          t.scale, t.lo, t.hi, t.loR, t.hiR ) );
    else
      check( transformBatch( ctx( ), kind, fwd, x, y, rows, cols, level, t.L, t.tw, t.scale,
          t.lo, t.hi, t.loR, t.hiR ) );
    return unpack( y, rows, cols );
  }

  /** Filter bank as passed to every call: {L, tw, scale} + 4 tap arrays. */
  static final class Taps {
    final int L, tw;
    final double scale;
    final double[ ] lo, hi, loR, hiR;

    Taps( Wavelet w, double scale ) {
      L = w.getMotherWavelength( );
      tw = w.getTransformWavelength( );
      lo = w.getScalingDeComposition( );
      hi = w.getWaveletDeComposition( );
      loR = w.getScalingReConstruction( );
      hiR = w.getWaveletReConstruction( );
      this.scale = scale;
    }
  }

  /**
   * The bank for wavelets the native path reproduces bit for bit, or null
   * (caller then runs the inherited Java code): classes that keep
   * Wavelet.forward/reverse (Wavelet.java:236-303), the BiOrthogonal family
   * (same math, BiOrthogonal.java:74-133) and Haar1Orthogonal (reverse x0.5,
   * Haar1Orthogonal.java:175-207).
   */
  static Taps tapsFor( Wavelet w ) {
    if( w == null || w.getMotherWavelength( ) > 64 )
      return null;
    if( w instanceof Haar1Orthogonal )
      return new Taps( w, 0.5 );
    if( w instanceof BiOrthogonal )
      return new Taps( w, 1.0 );
    try {
      Class< ? > f = w.getClass( ).getMethod( "forward", double[ ].class, int.class )
          .getDeclaringClass( );
      Class< ? > r = w.getClass( ).getMethod( "reverse", double[ ].class, int.class )
          .getDeclaringClass( );
      return ( f == Wavelet.class && r == Wavelet.class ) ? new Taps( w, 1.0 ) : null;
    } catch( NoSuchMethodException e ) {
      return null;
    }
  }

  /** Status -> the reference's exception types (SURVEY §8b). */
  static void check( int rc ) throws JWaveException {
    if( rc == OK )
      return;
    String msg = lastError( ctx( ) );
    switch( rc ) {
      case FAILURE:          throw new JWaveFailure( msg );
      case ILLEGAL_ARGUMENT: throw new IllegalArgumentException( msg );
      default:               throw new JWaveError( msg );
    }
  }

  // ---- natives (java/native/jwave_hip_jni.c) -------------------------------
  static native int ctxCreate( int device, long[ ] out );
  static native String lastError( long ctx );

  /** kind: 0 = FWT, 1 = WPT.  x and y are distinct arrays of length n. */
  static native int transform1d( long ctx, int kind, boolean forward, double[ ] x, double[ ] y,
      int level, int L, int tw, double scale, double[ ] lo, double[ ] hi, double[ ] loR,
      double[ ] hiR );

  static native int mctxCreate( int[ ] devices, long[ ] out );
  static native String mctxLastError( long mctx );

  /** transformBatch over the devices of a multi-context (jwv_m_*_batch_f64). */
  static native int transformBatchMulti( long mctx, int kind, boolean forward, double[ ] x,
      double[ ] y, int batch, int n, int level, int L, int tw, double scale, double[ ] lo,
      double[ ] hi, double[ ] loR, double[ ] hiR );

  /** transform2d over the devices of a multi-context (jwv_m_{fwt,wpt}2d_*):
   *  row blocks, one device-to-device exchange, column slabs. */
  static native int transform2dMulti( long mctx, int kind, boolean forward, double[ ] x,
      double[ ] y, int rows, int cols, int lvlM, int lvlN, int L, int tw, double scale,
      double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  /** forwardMODWT / inverseMODWT of `batch` signals: x = batch*n, wv =
   *  batch*(J+1)*n (jwv_m_modwt_*_batch_f64 / jwv_modwt_*_batch_f64). */
  static native int modwtBatchMulti( long mctx, boolean forward, double[ ] x, double[ ] wv,
      int batch, int n, int J, int L, int tw, double[ ] lo, double[ ] hi, double[ ] loR,
      double[ ] hiR );
  static native int modwtBatch( long ctx, boolean forward, double[ ] x, double[ ] wv, int batch,
      int n, int J, int L, int tw, double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  /** batch signals of length n, packed contiguously (ld = n). */
  static native int transformBatch( long ctx, int kind, boolean forward, double[ ] x,
      double[ ] y, int batch, int n, int level, int L, int tw, double scale, double[ ] lo,
      double[ ] hi, double[ ] loR, double[ ] hiR );

  /** Rows packed contiguously (rows*cols) by the caller. */
  static native int transform2d( long ctx, int kind, boolean forward, double[ ] x, double[ ] y,
      int rows, int cols, int lvlM, int lvlN, int L, int tw, double scale, double[ ] lo,
      double[ ] hi, double[ ] loR, double[ ] hiR );

  static native int transform3d( long ctx, int kind, boolean forward, double[ ] x, double[ ] y,
      int p, int q, int r, int lvlP, int lvlQ, int lvlR, int L, int tw, double scale,
      double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  /** ParallelTransform's 3-D reverse order: the P axis first, then the slices
   *  (ParallelTransform.java:183-216). */
  static native int transform3dPt( long ctx, int kind, double[ ] x, double[ ] y, int p, int q,
      int r, int lvlP, int lvlQ, int lvlR, int L, int tw, double scale, double[ ] lo,
      double[ ] hi, double[ ] loR, double[ ] hiR );

  /** wv = (J+1)*n doubles, rows W_1..W_J, V_J. */
  static native int modwt( long ctx, boolean forward, double[ ] x, double[ ] wv, int n, int J,
      int L, int tw, double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  /** AncientEgyptianDecomposition over FWT (kind 0) / WPT (kind 1), any length. */
  static native int aed( long ctx, int kind, boolean forward, double[ ] x, double[ ] y, int L,
      int tw, double scale, double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  /** mat = (log2 n + 1) * n doubles, row p = forward(x, p). */
  static native int decompose( long ctx, int kind, double[ ] x, double[ ] mat, int L, int tw,
      double scale, double[ ] lo, double[ ] hi, double[ ] loR, double[ ] hiR );

  static int t1( int kind, boolean fwd, double[ ] x, double[ ] y, int level, Taps t ) {
    return transform1d( ctx( ), kind, fwd, x, y, level, t.L, t.tw, t.scale, t.lo, t.hi, t.loR,
        t.hiR );
  }

  /** rows * cols doubles fit one Java array (the int product would
   *  overflow past 2^31 - 1; VMs cap arrays a few elements below that). */
  static boolean fitsArray( long rows, long cols ) {
    return rows * cols <= Integer.MAX_VALUE - 8;
  }

  static double[ ] pack( double[ ][ ] m ) {
    int rows = m.length, cols = rows == 0 ? 0 : m[ 0 ].length;
    if( !fitsArray( rows, cols ) )  // callers check first and keep the Java path
      throw new IllegalArgumentException( "HipNative#pack - " + rows + " x " + cols
          + " doubles exceed one Java array" );
    double[ ] out = new double[ rows * cols ];
    for( int i = 0; i < rows; i++ )
      System.arraycopy( m[ i ], 0, out, i * cols, cols );
    return out;
  }

  static boolean fits3d( double[ ][ ][ ] s ) {
    long P = s.length, Q = P == 0 ? 0 : s[ 0 ].length, R = Q == 0 ? 0 : s[ 0 ][ 0 ].length;
    return fitsArray( P * Q, R );
  }

  /** BasicTransform.forward|reverse(double[][], lvlM, lvlN) in one call: over
   *  the jwave.hip.devices GPUs when set (row blocks, one device-to-device
   *  exchange, column slabs: ParallelTransform.java:70-126's split), else on
   *  this thread's device.  The same bits either way. */
  static double[ ][ ] run2d( int kind, Taps t, boolean fwd, double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    int rows = m.length, cols = rows == 0 ? 0 : m[ 0 ].length;
    double[ ] x = pack( m ), y = new double[ x.length ];
    long mc = mctx( );
    if( mc != 0L )
      checkMulti( mc, transform2dMulti( mc, kind, fwd, x, y, rows, cols, lvlM, lvlN, t.L, t.tw,
          t.scale, t.lo, t.hi, t.loR, t.hiR ) );
    else
      check( transform2d( ctx( ), kind, fwd, x, y, rows, cols, lvlM, lvlN, t.L, t.tw, t.scale,
          t.lo, t.hi, t.loR, t.hiR ) );
    return unpack( y, rows, cols );
  }

  /** forwardMODWT of every signal (equal lengths) in one native call: over
   *  the jwave.hip.devices GPUs when set, else this thread's device.
   *  Returns [signal][level row][n]. */
  static double[ ][ ][ ] modwtForwardBatch( Taps t, double[ ][ ] signals, int J )
      throws JWaveException {
    int b = signals.length, n = b == 0 ? 0 : signals[ 0 ].length;
    double[ ] x = pack( signals ), wv = new double[ b * ( J + 1 ) * n ];
    long mc = mctx( );
    if( mc != 0L )
      checkMulti( mc, modwtBatchMulti( mc, true, x, wv, b, n, J, t.L, t.tw, t.lo, t.hi, t.loR,
          t.hiR ) );
    else
      check( modwtBatch( ctx( ), true, x, wv, b, n, J, t.L, t.tw, t.lo, t.hi, t.loR, t.hiR ) );
    double[ ][ ][ ] out = new double[ b ][ ][ ];
    for( int i = 0; i < b; i++ ) {
      out[ i ] = new double[ J + 1 ][ n ];
      for( int r = 0; r <= J; r++ )
        System.arraycopy( wv, ( i * ( J + 1 ) + r ) * n, out[ i ][ r ], 0, n );
    }
    return out;
  }

  /** inverseMODWT of every signal's [J+1][n] coefficients in one native call. */
  static double[ ][ ] modwtInverseBatch( Taps t, double[ ][ ][ ] c ) throws JWaveException {
    int b = c.length, J = c[ 0 ].length - 1, n = c[ 0 ][ 0 ].length;
    double[ ] wv = new double[ b * ( J + 1 ) * n ], x = new double[ b * n ];
    for( int i = 0; i < b; i++ )
      for( int r = 0; r <= J; r++ )
        System.arraycopy( c[ i ][ r ], 0, wv, ( i * ( J + 1 ) + r ) * n, n );
    long mc = mctx( );
    if( mc != 0L )
      checkMulti( mc, modwtBatchMulti( mc, false, x, wv, b, n, J, t.L, t.tw, t.lo, t.hi, t.loR,
          t.hiR ) );
    else
      check( modwtBatch( ctx( ), false, x, wv, b, n, J, t.L, t.tw, t.lo, t.hi, t.loR, t.hiR ) );
    return unpack( x, b, n );
  }

  /** BasicTransform.forward|reverse(double[][][], lvlP, lvlQ, lvlR) in one
   *  call; pt: ParallelTransform's reverse order (P axis first). */
  static double[ ][ ][ ] run3d( int kind, Taps t, boolean fwd, boolean pt, double[ ][ ][ ] s,
      int lp, int lq, int lr ) throws JWaveException {
    int P = s.length, Q = P == 0 ? 0 : s[ 0 ].length, R = Q == 0 ? 0 : s[ 0 ][ 0 ].length;
    double[ ] x = new double[ P * Q * R ];
    for( int i = 0; i < P; i++ )
      for( int j = 0; j < Q; j++ )
        System.arraycopy( s[ i ][ j ], 0, x, ( i * Q + j ) * R, R );
    double[ ] y = new double[ x.length ];
    if( pt )
      check( transform3dPt( ctx( ), kind, x, y, P, Q, R, lp, lq, lr, t.L, t.tw, t.scale, t.lo,
          t.hi, t.loR, t.hiR ) );
    else
      check( transform3d( ctx( ), kind, fwd, x, y, P, Q, R, lp, lq, lr, t.L, t.tw, t.scale,
          t.lo, t.hi, t.loR, t.hiR ) );
    double[ ][ ][ ] out = new double[ P ][ Q ][ R ];
    for( int i = 0; i < P; i++ )
      for( int j = 0; j < Q; j++ )
        System.arraycopy( y, ( i * Q + j ) * R, out[ i ][ j ], 0, R );
    return out;
  }

  static double[ ][ ] unpack( double[ ] a, int rows, int cols ) {
    double[ ][ ] m = new double[ rows ][ cols ];
    for( int i = 0; i < rows; i++ )
      System.arraycopy( a, i * cols, m[ i ], 0, cols );
    return m;
  }
}

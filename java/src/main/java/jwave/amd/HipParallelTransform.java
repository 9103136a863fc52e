/*
 * HipParallelTransform — ParallelTransform (ParallelTransform.java:23-403)
 * around a HipFastWaveletTransform / HipWaveletPacketTransform (any
 * HipTransform).
 *
 * The reference forks RowTransformTask / ColumnTransformTask /
 * Space3DTransformTask, which call the wrapped transform once per row, column
 * or line (:247-263, :307-330, :380-397): around a Hip transform that is one
 * native call (and one PCIe round trip) per line, 16,384 of them for an
 * 8192 x 8192 matrix.  Here each 2-D / 3-D call is ONE native call with the
 * reference's result:
 *  - 2-D forward / reverse and the 3-D forward run in the order the tasks
 *    use, which is the wrapped transform's own BasicTransform order (rows with
 *    lvlN then columns with lvlM; slices then the P axis);
 *  - the 3-D reverse runs the P axis first, then the slices (:183-216), which
 *    BasicTransform.reverse does the other way round: HipNative.transform3dPt.
 * Matrices below MIN_PARALLEL_SIZE go to the wrapped transform (:73-76), as in
 * the reference.  Errors carry the reference's "Error in parallel .." prefix.
 * 1-D calls delegate, as ParallelTransform's do.  A wrapped transform the
 * native path does not cover (no taps) keeps the reference's ForkJoin code.
 *
 * Drop-in: new ParallelTransform( new HipFastWaveletTransform( w ) ) keeps
 * working (per-line native calls); HipParallelTransform.of( t ) returns this
 * class for Hip transforms and a plain ParallelTransform otherwise.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.BasicTransform;
import jwave.transforms.ParallelTransform;
import jwave.tools.MathToolKit;

public class HipParallelTransform extends ParallelTransform {

  private static final int MIN_PARALLEL_SIZE = 16;  // ParallelTransform.java:28
  private final BasicTransform _t;
  private final HipTransform _hip;

  public HipParallelTransform( HipFastWaveletTransform transform ) {
    this( (BasicTransform)transform, transform, -1 );
  }

  public HipParallelTransform( HipWaveletPacketTransform transform ) {
    this( (BasicTransform)transform, transform, -1 );
  }

  public HipParallelTransform( HipFastWaveletTransform transform, int parallelism ) {
    this( (BasicTransform)transform, transform, parallelism );
  }

  public HipParallelTransform( HipWaveletPacketTransform transform, int parallelism ) {
    this( (BasicTransform)transform, transform, parallelism );
  }

  private HipParallelTransform( BasicTransform t, HipTransform hip, int parallelism ) {
    super( t, parallelism > 0 ? parallelism
        : java.util.concurrent.ForkJoinPool.getCommonPoolParallelism( ) );
    _t = t;
    _hip = hip;
  }

  /** The parallel wrapper for t: this class around Hip transforms, the
   *  reference's ParallelTransform otherwise. */
  public static ParallelTransform of( BasicTransform t ) {
    if( t instanceof HipTransform )
      return new HipParallelTransform( t, (HipTransform)t, -1 );
    return new ParallelTransform( t );
  }

  private boolean nativeOk( double[ ][ ] m ) {
    return _hip.taps( ) != null
        && HipNative.fitsArray( m.length, m.length == 0 ? 0 : m[ 0 ].length );
  }

  private boolean small( double[ ][ ] m ) {
    return m.length < MIN_PARALLEL_SIZE || m[ 0 ].length < MIN_PARALLEL_SIZE;
  }

  // the reference's tasks wrap the cause in a RuntimeException (ParallelTransform.java:259-269),
  // whose message is the cause's Throwable.toString(); a ForkJoin re-wrap on a
  // pool worker ("java.lang.RuntimeException: ...") is scheduling-dependent and
  // not reproduced
  private static JWaveException wrap( String what, JWaveException e ) {
    return new JWaveException( "Error in parallel " + what + " transform: " + e.toString( ) );
  }

  @Override public double[ ][ ] forward( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( !nativeOk( m ) )
      return super.forward( m, lvlM, lvlN );
    if( small( m ) )
      return _t.forward( m, lvlM, lvlN );
    try {
      return _t.forward( m, lvlM, lvlN );  // one native call (run2d)
    } catch( JWaveException e ) {
      throw wrap( "2D forward", e );
    }
  }

  @Override public double[ ][ ] reverse( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( !nativeOk( m ) )
      return super.reverse( m, lvlM, lvlN );
    if( small( m ) )
      return _t.reverse( m, lvlM, lvlN );
    try {
      return _t.reverse( m, lvlM, lvlN );
    } catch( JWaveException e ) {
      throw wrap( "2D reverse", e );
    }
  }

  private boolean nativeOk( double[ ][ ][ ] s ) {
    long P = s.length, Q = P == 0 ? 0 : s[ 0 ].length, R = Q == 0 ? 0 : s[ 0 ][ 0 ].length;
    return _hip.taps( ) != null && HipNative.fitsArray( P * Q, R );
  }

  @Override public double[ ][ ][ ] forward( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( !nativeOk( s ) )
      return super.forward( s, lvlP, lvlQ, lvlR );
    try {
      return _t.forward( s, lvlP, lvlQ, lvlR );  // one native call (run3d)
    } catch( JWaveException e ) {
      throw wrap( "3D forward", e );
    }
  }

  @Override public double[ ][ ][ ] reverse( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( !nativeOk( s ) )
      return super.reverse( s, lvlP, lvlQ, lvlR );
    try {
      return HipNative.run3d( _hip.kind( ), _hip.taps( ), false, true, s, lvlP, lvlQ, lvlR );
    } catch( JWaveException e ) {
      throw wrap( "3D reverse", e );
    }
  }

  // default-level overloads resolve through MathToolKit.getExponent, as the
  // reference's do (ParallelTransform.java:62-66, 96-100, 128-134, 175-181)
  @Override public double[ ][ ] forward( double[ ][ ] m ) throws JWaveException {
    return forward( m, MathToolKit.getExponent( m.length ),
        MathToolKit.getExponent( m[ 0 ].length ) );
  }

  @Override public double[ ][ ] reverse( double[ ][ ] m ) throws JWaveException {
    return reverse( m, MathToolKit.getExponent( m.length ),
        MathToolKit.getExponent( m[ 0 ].length ) );
  }
}
